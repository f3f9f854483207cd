#!/bin/bash
# Round 5: the replica race measured (host p50 per block + kernel trace of the octet kernels), then the lazy-reduction
# C2 A/B on the product build and charon_amd/libhipbls_lazy.so, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/race_trace
cd $R
export PYTHONPATH=$R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/race_trace -o run -- python3 -u scripts/race_trace.py 100 > $O/race_trace/host.jsonl 2> $O/race_trace/err.log || { echo "race trace failed"; tail -20 $O/race_trace/err.log; exit 1; }
cat $O/race_trace/host.jsonl
C2="--steps 5 --warmup 1 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $C2 > $O/r05d_c2_prod$k.json 2> $O/r05d_c2_prod$k.err || { echo "c2 prod failed"; tail -20 $O/r05d_c2_prod$k.err; exit 1; }
  HIPBLS_LIB=$R/charon_amd/libhipbls_lazy.so timeout -k 10 300 python -u bench.py $C2 > $O/r05d_c2_lazy$k.json 2> $O/r05d_c2_lazy$k.err || { echo "c2 lazy failed"; tail -20 $O/r05d_c2_lazy$k.err; exit 1; }
  for f in $O/r05d_c2_prod$k.json $O/r05d_c2_lazy$k.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
done
