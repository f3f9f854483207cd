#!/bin/bash
# Round 4: kernel timelines of C3 (sigagg in one call) and of the n = 1 drop-in latency loop.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
A3="--c2-items 4096 --steps 1 --warmup 0 --tagg-steps 3 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_c3 -o c3 -- python3 -u bench.py $A3 > $O/tr_c3.json 2> $O/tr_c3.err || { echo "c3 trace failed"; tail -20 $O/tr_c3.err; exit 1; }
AL="--c2-items 4096 --steps 1 --warmup 0 --tagg-steps 1 --tagg-groups 64 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 40 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_lat -o lat -- python3 -u bench.py $AL > $O/tr_lat.json 2> $O/tr_lat.err || { echo "lat trace failed"; tail -20 $O/tr_lat.err; exit 1; }
find $O/tr_c3 $O/tr_lat -name "*.csv" | head
