#!/bin/bash
# Round 4: the sigagg key-side loop ahead of the aggregate -- its GPU tests (fused == two calls in every layout,
# full-size C3 bytes, multi-context) and a C2/C3-only bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r04.py "tests/test_gpu_r02.py::test_threshold_aggregate_verify_fused_equals_two_calls" tests/test_gpu_multidev.py > $O/r04c_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04c_pytest.log; exit 1; }
tail -8 $O/r04c_pytest.log
timeout -k 10 300 python -u bench.py --rlc-node-validators 0 --c5 0 --latency-calls 50 --cpu-sample 0 --keys 0 > $O/r04c_bench.json 2> $O/r04c_bench.err || { echo "bench failed"; tail -30 $O/r04c_bench.err; exit 1; }
cat $O/r04c_bench.json
