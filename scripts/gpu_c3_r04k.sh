#!/bin/bash
# Round 4: C3 with the key prep dispatched ahead of the scaling, three short runs of 5 steps each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
ARGS="--c2-items 4096 --steps 1 --warmup 0 --tagg-steps 5 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0"
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py $ARGS > $O/c3k_$k.json 2> $O/c3k_$k.err || { echo "run $k failed"; tail -20 $O/c3k_$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/c3k_$k.json'))
print('run $k', d['threshold_aggregates_per_s'], d['threshold_aggregate_kernel_avg_ms'])"
done
