#!/bin/bash
# Round 4: the eight-lane Verify (verify_lat.hip, split Fp2 products) -- layout parity tests first, then the drop-in
# latency (n = 1 calls) and a per-layout batch sweep.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lg2.py > $O/r04f_lg2.log 2>&1 || { echo "lg2 tests failed"; tail -40 $O/r04f_lg2.log; exit 1; }
tail -3 $O/r04f_lg2.log
timeout -k 10 300 python -u scripts/latency_sweep.py > $O/r04f_lat.json 2> $O/r04f_lat.err || { echo "latency sweep failed"; tail -30 $O/r04f_lat.err; exit 1; }
cat $O/r04f_lat.json
