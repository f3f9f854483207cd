#!/bin/bash
# Round 5 at HEAD: the whole GPU suite, smoke(), the default bench, then the same bench under rocprofv3 --kernel-trace
# --stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/final_prof
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/final_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/final_suite.log; exit 1; }
tail -1 $O/final_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/final_smoke.log; exit 1; }
tail -1 $O/final_smoke.log
timeout -k 10 560 python -u bench.py > $O/final_bench.json 2> $O/final_bench.err || { echo "bench failed"; tail -30 $O/final_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/final_bench.json'))
print('C2', d['value'], d['roofline']['frac'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'])
print('lat', d['drop_in_latency'])
print('host', d['host_path'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/final_prof -o run -- python3 -u $R/bench.py > $O/final_bench_profiled.json 2> $O/final_bench_profiled.err || { echo "profiled bench failed"; tail -30 $O/final_bench_profiled.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/final_bench_profiled.json')); print('profiled C2', d['value'], d['roofline']['kernel_avg_ms'], d['drop_in_latency']['p50_ms'])"
