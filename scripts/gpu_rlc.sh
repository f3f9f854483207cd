#!/bin/bash
# Quick GPU iteration on the RLC path: its parity tests, then the bench without C3 / cpu baseline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_rlc.py -x -v --timeout 120 --timeout-method thread > $O/pytest_rlc.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_rlc.log; exit 1; }
tail -3 $O/pytest_rlc.log
timeout -k 10 300 python -u bench.py --steps 3 --tagg-groups 0 --cpu-sample 0 ${BENCH_ARGS:-} > $O/bench_rlc.json 2> $O/bench_rlc.err || { echo "bench failed"; tail -30 $O/bench_rlc.err; exit 1; }
cat $O/bench_rlc.json
