#!/bin/bash
# Round 5: which part of the default bench moves C5 (270 ms in a C4(i)-only run, 280 ms in the default run): the
# C4(i)-only run again, then with the pubshare table loaded first (--keys 1), then after all four C4 variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd $R
B="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 1 --latency-calls 0 --host-path 0 --rlc-steps 3"
for v in "k0_i:--keys 0 --rlc-variants i" "k1_i:--keys 1 --rlc-variants i" "k0_all:--keys 0"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python -u bench.py $B $args > $O/r05q_$tag.json 2> $O/r05q_$tag.err || { echo "$tag failed"; tail -20 $O/r05q_$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/r05q_$tag.json')); print('$tag', 'C5', d['full_slot_mix']['ms_per_slot'], {k: v.get('ms_per_batch') for k, v in d['rlc_batch_verify'].items() if isinstance(v, dict)})"
done
