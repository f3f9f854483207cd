#!/bin/bash
# Kernel timeline of the RLC path (C4 shard) for the overlap analysis: rocprofv3 kernel trace only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o rlc -- python3 $R/bench.py --c2-items 1024 --steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 32768 --rlc-steps 2 > $O/trace_bench.json 2> $O/trace_bench.err || { echo "trace failed"; tail -20 $O/trace_bench.err; exit 1; }
ls -R $O/trace | head
