#!/bin/bash
# A/B of compile-time variants on the C4 workloads (1M-partial node batch: windows, committee roots, all-valid batch
# check): the in-tree build, then each scratch_ab/libhipbls_<v>.so given on the command line (HIPBLS_LIB).
set -o pipefail
mkdir -p gpurun_out
ARGS="--c2-items 4096 --tagg-groups 0 --c5 0 --keys 0 --cpu-sample 0 --steps 2 --warmup 1 --rlc-steps 3"
timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/c4_base.json 2> gpurun_out/c4_base.err || exit 1
for v in "$@"; do
  HIPBLS_LIB=scratch_ab/libhipbls_$v.so timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/c4_$v.json 2> gpurun_out/c4_$v.err || exit 1
done
for f in gpurun_out/c4_*.json; do
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))['rlc_batch_verify']
print(sys.argv[1])
for k,v in d.items():
    if isinstance(v,dict): print('  ',k, v['verified_partial_sigs_per_s'], v['ms_per_batch'], v.get('kernel_avg_ms'))
" $f
done
