#!/bin/bash
# Round 4, full check at HEAD: the whole GPU suite (one pytest process), smoke, the default bench, and the kernel
# trace + stats of the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/ > $O/r04g_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04g_pytest.log; exit 1; }
tail -4 $O/r04g_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r04g_smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/r04g_smoke.log; exit 1; }
tail -3 $O/r04g_smoke.log
timeout -k 10 500 python -u bench.py > $O/r04g_bench.json 2> $O/r04g_bench.err || { echo "bench failed"; tail -30 $O/r04g_bench.err; exit 1; }
cat $O/r04g_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04g -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --latency-calls 0 > $O/prof_r04g_bench.json 2> $O/prof_r04g_bench.err || { echo "trace failed"; tail -20 $O/prof_r04g_bench.err; exit 1; }
find $O/prof_r04g -name '*stats*'
