#!/bin/bash
# Round 5: C5's partial last window waves go to the per-item checks: the RLC / config / small-order tests and the new
# round-5 tests, then C4(i) + C5 (windows, AUTO, failed batch check) twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
export PYTHONPATH=$R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r05.py tests/test_gpu_rlc.py tests/test_gpu_rlcb.py tests/test_gpu_configs.py tests/test_gpu_small_order.py > $O/r05u_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05u_first.log; exit 1; }
tail -1 $O/r05u_first.log
B="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 1 --keys 0 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 3"
for k in 1 2; do
timeout -k 10 400 python -u bench.py $B > $O/r05u_c5_$k.json 2> $O/r05u_c5_$k.err || { echo "c5 failed"; tail -20 $O/r05u_c5_$k.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05u_c5_$k.json')); r=d['rlc_batch_verify']['i_root_per_validator']; c=d['full_slot_mix']
print('C4i', r['ms_per_batch'], r['failed_batch_check_ms_per_batch'], r['auto_mode_amortized_ms_per_batch'], 'C5', c['ms_per_slot'], c['failed_batch_check_ms_per_slot'], c['auto_mode_amortized_ms_per_slot'])"
done
