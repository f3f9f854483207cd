#!/bin/bash
# Round 5: the race with global sc1 polls: the layout-parity, round-5 and queue tests, then the race trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/race_trace3
cd $R
export PYTHONPATH=$R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lg2.py tests/test_gpu_r05.py "tests/test_gpu_r02.py::test_queue_concurrent_single_verifies_equal_batch" > $O/r05e_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05e_tests.log; exit 1; }
tail -1 $O/r05e_tests.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/race_trace3 -o run -- python3 -u scripts/race_trace.py 100 > $O/race_trace3/host.jsonl 2> $O/race_trace3/err.log || { echo "race trace failed"; tail -20 $O/race_trace3/err.log; exit 1; }
cat $O/race_trace3/host.jsonl
