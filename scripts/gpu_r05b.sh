#!/bin/bash
# Round 5: replica race on the n = 1 path + the last RLC sub-batch's fallback on lane pairs: the layout-parity and
# queue tests first, then the whole GPU suite, then the default bench once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_lg2.py tests/test_gpu_r05.py tests/test_gpu_r04.py > $O/r05b_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05b_first.log; exit 1; }
tail -1 $O/r05b_first.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/r05b_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05b_suite.log; exit 1; }
tail -1 $O/r05b_suite.log
timeout -k 10 500 python -u bench.py > $O/r05b_bench.json 2> $O/r05b_bench.err || { echo "bench failed"; tail -30 $O/r05b_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05b_bench.json'))
print('C2', d['value'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'])
print('lat', d['drop_in_latency'])
print('host', d['host_path'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'), v.get('items_fallback'))"
