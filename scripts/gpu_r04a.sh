#!/bin/bash
# Round 4, first box: the new sigagg-bytes / C1 tests, the multi-context test (shared device streams), smoke, then
# the default bench (C3 now asserts the aggregate bytes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r04.py tests/test_gpu_multidev.py > $O/r04a_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04a_pytest.log; exit 1; }
tail -8 $O/r04a_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04a_smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/r04a_smoke.log; exit 1; }
cat $O/r04a_smoke.log
timeout -k 10 400 python -u bench.py > $O/r04a_bench.json 2> $O/r04a_bench.err || { echo "bench failed"; tail -30 $O/r04a_bench.err; exit 1; }
cat $O/r04a_bench.json
