#!/bin/bash
# Round 4: batch-wide RLC check with the chunk kernel at one wave per SIMD (S-factor in the final pair) and AoS MSM
# points: the RLC GPU tests, then the C4 part of the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rlcb.py tests/test_gpu_rlc.py tests/test_gpu_configs.py > $O/r04d_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04d_pytest.log; exit 1; }
tail -5 $O/r04d_pytest.log
timeout -k 10 400 python -u bench.py --c2-items 40960 --tagg-groups 0 --latency-calls 0 --cpu-sample 0 > $O/r04d_bench.json 2> $O/r04d_bench.err || { echo "bench failed"; tail -30 $O/r04d_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04d_bench.json'))
for k,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(k, v['ms_per_batch'], v['verified_partial_sigs_per_s'], v.get('kernel_avg_ms'))
print('c5', d.get('full_slot_mix',{}).get('ms_per_slot'))"
