#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel stats.  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof failed"; tail -30 $O/prof_bench.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cat {} \;
