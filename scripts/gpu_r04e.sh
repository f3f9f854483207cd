#!/bin/bash
# Round 4: the G1 MSM per committee root in the batch-wide RLC check (g1msm.h): its GPU tests, the RLC/C4 GPU
# tests, then the C4 part of the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_r04.py -k g1_msm > $O/r04e_g1.log 2>&1 || { echo "g1 pytest failed"; tail -40 $O/r04e_g1.log; exit 1; }
tail -4 $O/r04e_g1.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rlcb.py tests/test_gpu_configs.py > $O/r04e_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04e_pytest.log; exit 1; }
tail -5 $O/r04e_pytest.log
timeout -k 10 400 python -u bench.py --c2-items 40960 --tagg-groups 0 --latency-calls 0 --cpu-sample 0 > $O/r04e_bench.json 2> $O/r04e_bench.err || { echo "bench failed"; tail -30 $O/r04e_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04e_bench.json'))
for k,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(k, v['ms_per_batch'], v['verified_partial_sigs_per_s'], v.get('kernel_avg_ms'))
print('c5', d.get('full_slot_mix',{}).get('ms_per_slot'))"
