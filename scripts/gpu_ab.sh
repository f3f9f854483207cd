#!/bin/bash
# Quick A/B after a kernel change: C2 bench only, then the -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
python3 -c "
import json;d=json.load(open('gpurun_out/ab.json'))
print('C2', d['value'], d['ms_per_step'], 'frac', d.get('roofline',{}).get('frac'), 'C3', d['threshold_aggregates_per_s'], 'keys', d['verified_partial_sigs_per_s_pubshare_table'])
r=d.get('rlc_batch_verify',{})
for k,v in r.items():
  if isinstance(v,dict): print(k, v['verified_partial_sigs_per_s'], v['kernel_avg_ms'])
if 'full_slot_mix' in d: print('C5', d['full_slot_mix']['verified_partial_sigs_per_s'])
"
tail -3 gpurun_out/pytest_gpu.log
exit $rc
