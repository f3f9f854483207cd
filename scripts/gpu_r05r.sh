#!/bin/bash
# Round 5: what a failed batch-wide check costs on C4(i) (1 % invalid): the bench's variant i alone (windows, AUTO,
# then forced BATCH) and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/c4trace4
cd $R
B="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 3"
timeout -k 10 400 python -u bench.py $B > $O/r05r.json 2> $O/r05r.err || { echo "bench failed"; tail -20 $O/r05r.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05r.json')); r=d['rlc_batch_verify']['i_root_per_validator']
print({k: r[k] for k in ('ms_per_batch', 'auto_mode_ms_per_batch', 'failed_batch_check_ms_per_batch', 'auto_mode_amortized_ms_per_batch')})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c4trace4 -o run -- python3 $R/bench.py $B > $O/c4trace4/out.json 2> $O/c4trace4/err.log || { echo "trace failed"; tail -20 $O/c4trace4/err.log; exit 1; }
echo done
