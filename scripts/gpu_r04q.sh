#!/bin/bash
# Round 4: submission queue with a 50 us idle gather window and 20 us completion polling -- the queue tests, then
# the default bench (n = 1 drop-in latency).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_r02.py tests/test_gpu_r03.py tests/test_gpu_small_order.py tests/test_gpu_r04.py > $O/r04q_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04q_pytest.log; exit 1; }
tail -3 $O/r04q_pytest.log
timeout -k 10 500 python -u bench.py > $O/r04q_bench.json 2> $O/r04q_bench.err || { echo "bench failed"; tail -30 $O/r04q_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04q_bench.json'))
print('C2', d['value'], 'lat', d['drop_in_latency'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'])"
