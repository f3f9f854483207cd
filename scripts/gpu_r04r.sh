#!/bin/bash
# Round 4: sub[1] at high stream priority -- the RLC batch-check tests, then the default bench twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_rlcb.py tests/test_gpu_multidev.py > $O/r04r_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04r_pytest.log; exit 1; }
tail -2 $O/r04r_pytest.log
for k in 1 2; do
timeout -k 10 500 python -u bench.py --latency-calls 0 --cpu-sample 0 > $O/r04r_bench$k.json 2> $O/r04r_bench$k.err || { echo "bench failed"; tail -30 $O/r04r_bench$k.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04r_bench$k.json'))
print('C2', d['value'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v['ms_per_batch'])"
done
