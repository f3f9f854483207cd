#!/bin/bash
# A/B of library builds: for each charon_amd/libhipbls_<name>.so given, install it as libhipbls.so and run the full
# bench once (each run under its own time limit); the original library is restored at the end.
set -o pipefail
mkdir -p gpurun_out
cp charon_amd/libhipbls.so gpurun_out/.lib_orig.so
rc=0
for v in base "$@"; do
  if [ "$v" != base ]; then cp charon_amd/libhipbls_$v.so charon_amd/libhipbls.so; fi
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "variant $v failed"; rc=1; break; }
  python3 -c "
import json,sys;d=json.load(open('gpurun_out/var_$v.json'))
r=d['rlc_batch_verify']
print('$v', 'C2', d['value'], d['ms_per_step'], 'C3', d['threshold_aggregates_per_s'], 'C4i', r['i_root_per_validator']['verified_partial_sigs_per_s'], 'C4all', r['i_all_valid']['verified_partial_sigs_per_s'], 'C5', d['full_slot_mix']['verified_partial_sigs_per_s'])"
done
cp gpurun_out/.lib_orig.so charon_amd/libhipbls.so
exit $rc
