#!/bin/bash
# Round 4: kernel stats of the C4 all-valid variants (MSM stages) under rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R
A="--c2-items 4096 --steps 1 --warmup 0 --tagg-groups 64 --tagg-steps 1 --rlc-variants all_valid,ii_all_valid --rlc-steps 3 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_c4 -o c4 -- python3 -u bench.py $A > $O/tr_c4.json 2> $O/tr_c4.err || { echo "c4 trace failed"; tail -20 $O/tr_c4.err; exit 1; }
find $O/tr_c4 -name "*.csv" | head
