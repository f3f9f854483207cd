#!/bin/bash
# Round 5: replica counts 8 / 16 / 32 on the n = 1 path (kernel trace), then the queued n = 1 latency with the
# adaptive gather window (bench latency section only, twice).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/race_trace8
cd $R
export PYTHONPATH=$R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/race_trace8 -o run -- python3 -u scripts/race_trace.py 100 8,16,32,8,16,32 > $O/race_trace8/host.jsonl 2> $O/race_trace8/err.log || { echo "race trace failed"; tail -20 $O/race_trace8/err.log; exit 1; }
cat $O/race_trace8/host.jsonl
L="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --host-path 0 --latency-calls 1000"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $L > $O/r05k_lat$k.json 2> $O/r05k_lat$k.err || { echo "latency bench failed"; tail -20 $O/r05k_lat$k.err; exit 1; }
  python3 -c "import json; print(json.load(open('$O/r05k_lat$k.json'))['drop_in_latency'])"
done
