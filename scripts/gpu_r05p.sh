#!/bin/bash
# Round 5: kernel trace of C4(i) (windows, 1 % invalid) on the wire-format call and on the pubshare-table call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/c4trace3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c4trace3 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 0 --keys 1 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 2 > $O/c4trace3/out.json 2> $O/c4trace3/err.log || { echo "trace failed"; tail -20 $O/c4trace3/err.log; exit 1; }
echo done
