#!/bin/bash
# Round 4: the quad compressed squaring with distributed additions -- unit + layout + RLC/multi-context tests, then
# the C3 A/B against the worktree build and the latency sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_units.py tests/test_gpu_lg2.py tests/test_gpu_rlcb.py tests/test_gpu_multidev.py tests/test_gpu_r02.py > $O/r04h_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04h_pytest.log; exit 1; }
tail -3 $O/r04h_pytest.log
bash scripts/ab_c3.sh || exit 1
timeout -k 10 300 python -u scripts/latency_sweep.py > $O/r04h_lat.json 2> $O/r04h_lat.err || { echo "latency sweep failed"; tail -30 $O/r04h_lat.err; exit 1; }
cat $O/r04h_lat.json
