#!/bin/bash
# Round 5: kernel trace of the C4(i)-only bench with the pubshare table loaded (--keys 1), where C5 measured 358 ms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/c5trace2
B="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 1 --keys 1 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 3"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $O/c5trace2 -o run -- python3 $R/bench.py $B > $O/c5trace2/out.json 2> $O/c5trace2/err.log || { echo "trace failed"; tail -20 $O/c5trace2/err.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c5trace2/out.json')); r=d['rlc_batch_verify']['i_root_per_validator']
c=d['full_slot_mix']; print('C5', c['ms_per_slot'], c['failed_batch_check_ms_per_slot'], c['auto_mode_amortized_ms_per_slot'], {k: r[k] for k in ('ms_per_batch', 'auto_mode_ms_per_batch', 'failed_batch_check_ms_per_batch')})"
