#!/bin/bash
# Round 5: the prep's latency cuts (word-assembled expand_message for 32-byte roots, the cofactor clearing's additions
# on the quad, twin-lane right-to-left square roots) and denser race polls in the final exponentiation: the octet
# layout / race / RLC-tail / unit tests first, then the whole suite, the latency parts probe and the race trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/race_trace7
cd $R
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lg2.py tests/test_gpu_r05.py tests/test_gpu_units.py tests/test_gpu_rlcb.py > $O/r05j_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05j_first.log; exit 1; }
tail -1 $O/r05j_first.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/r05j_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05j_suite.log; exit 1; }
tail -1 $O/r05j_suite.log
timeout -k 10 120 charon_amd/tools/lat_parts_probe 8 > $O/lat_parts_8_j.txt || { echo "probe failed"; exit 1; }
cat $O/lat_parts_8_j.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/race_trace7 -o run -- python3 -u scripts/race_trace.py 100 > $O/race_trace7/host.jsonl 2> $O/race_trace7/err.log || { echo "race trace failed"; tail -20 $O/race_trace7/err.log; exit 1; }
cat $O/race_trace7/host.jsonl
