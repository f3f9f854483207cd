#!/bin/bash
# Round 5: the RLC fallback re-checks failed windows' items from the stored [r] pk, [r] sig (no decompression): the
# RLC / config / small-order tests, the whole suite, then C4(i) (windows, 1 % invalid) twice with its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/c4trace2
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rlc.py tests/test_gpu_rlcb.py tests/test_gpu_configs.py tests/test_gpu_small_order.py > $O/r05o_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05o_first.log; exit 1; }
tail -1 $O/r05o_first.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/r05o_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05o_suite.log; exit 1; }
tail -1 $O/r05o_suite.log
C4="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 1 --keys 0 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 3"
timeout -k 10 400 python -u bench.py $C4 > $O/r05o_c4.json 2> $O/r05o_c4.err || { echo "c4 failed"; tail -20 $O/r05o_c4.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05o_c4.json')); r=d['rlc_batch_verify']['i_root_per_validator']; print('C4i', r['ms_per_batch'], r['items_fallback'], r['kernel_avg_ms'], 'C5', d['full_slot_mix']['ms_per_slot'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c4trace2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 2 > $O/c4trace2/out.json 2> $O/c4trace2/err.log || { echo "trace failed"; exit 1; }
