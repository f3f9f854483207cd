#!/bin/bash
# A/B on one box: C4(i) all-valid with the pre-G1-MSM build (worktree ab_old at f8165bf) and HEAD, twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
ARGS="--c2-items 4096 --steps 1 --warmup 0 --tagg-groups 0 --rlc-variants all_valid --rlc-steps 3 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0"
for k in 1 2; do
  for t in old new; do
    if [ $t = old ]; then D=$R/ab_old; else D=$R; fi
    (cd $D && timeout -k 10 300 python -u bench.py $ARGS > $O/ab_$t$k.json 2> $O/ab_$t$k.err) || { echo "$t$k failed"; tail -20 $O/ab_$t$k.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_$t$k.json'))['rlc_batch_verify']['i_all_valid']
print('$t$k', d['ms_per_batch'], {k: v for k, v in d['kernel_avg_ms'].items() if k.startswith('rlcb')})"
  done
done
