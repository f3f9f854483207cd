#!/bin/bash
# Round 5: the default bench at HEAD, then the same command under rocprofv3 --kernel-trace --stats (the roofline's
# k_verify_fused average from HIP events must agree with the trace's).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/bench_prof
cd $R
timeout -k 10 560 python -u bench.py > $O/r05_bench.json 2> $O/r05_bench.err || { echo "bench failed"; tail -30 $O/r05_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05_bench.json'))
print('C2', d['value'], d['roofline']['frac'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'])
print('lat', d['drop_in_latency'])
print('host', d['host_path'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_prof -o run -- python3 -u $R/bench.py > $O/r05_bench_profiled.json 2> $O/r05_bench_profiled.err || { echo "profiled bench failed"; tail -30 $O/r05_bench_profiled.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05_bench_profiled.json')); print('profiled C2', d['value'], d['roofline'])"
