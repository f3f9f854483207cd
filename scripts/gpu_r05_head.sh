#!/bin/bash
# Round 5 at HEAD, short form: the whole GPU suite, smoke(), then the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/head_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/head_suite.log; exit 1; }
tail -1 $O/head_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/head_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/head_smoke.log; exit 1; }
tail -1 $O/head_smoke.log
timeout -k 10 560 python -u bench.py > $O/head_bench.json 2> $O/head_bench.err || { echo "bench failed"; tail -30 $O/head_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/head_bench.json'))
print('C2', d['value'], d['roofline']['frac'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix'])
print('lat', d['drop_in_latency']['p50_ms'], d['drop_in_latency']['serial_verifies_per_s'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'), v.get('verified_partial_sigs_per_s_pubshare_table'), v.get('auto_mode_amortized_ms_per_batch'))"
