#!/bin/bash
# Round 5: the scratch fix (reserve at init, StreamJoin for priority streams) -- the new tests first, then the
# whole GPU suite, then the default bench once.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_r05.py > $O/r05a_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/r05a_new.log; exit 1; }
grep -E "scratch:|priority streams:|queue worker:|passed|failed" $O/r05a_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests > $O/r05a_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05a_suite.log; exit 1; }
tail -2 $O/r05a_suite.log
timeout -k 10 500 python -u bench.py > $O/r05a_bench.json 2> $O/r05a_bench.err || { echo "bench failed"; tail -30 $O/r05a_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05a_bench.json'))
print('C2', d['value'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'], 'lat', d['drop_in_latency'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'))"
