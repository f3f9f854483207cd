#!/bin/bash
# A/B on one box: C3 (10,000 x 7-of-10 sigagg in one call) with the worktree build ab_old and HEAD, twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
ARGS="--c2-items 4096 --steps 1 --warmup 0 --tagg-steps 5 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0"
for k in 1 2; do
  for t in old new; do
    if [ $t = old ]; then D=$R/ab_old; else D=$R; fi
    (cd $D && timeout -k 10 300 python -u bench.py $ARGS > $O/ab3_$t$k.json 2> $O/ab3_$t$k.err) || { echo "$t$k failed"; tail -20 $O/ab3_$t$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab3_$t$k.json'))
print('$t$k', d['threshold_aggregates_per_s'], d['threshold_aggregate_kernel_avg_ms'])"
  done
done
