#!/bin/bash
# Round 5: FastAggregateVerify for a few groups on the octet prep + sixteen-lane check: the FAV tests (new layout test,
# parity, small order, the 512-key sync-committee case), the whole suite, then C5 (and C4(i)) with the kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/c5trace3
cd $R
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_r05.py::test_fav_octet_and_sixteen_lane_layouts_match_fav_batch tests/test_gpu_parity.py tests/test_gpu_small_order.py tests/test_gpu_r02.py tests/test_gpu_lg2.py > $O/r05t_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05t_first.log; exit 1; }
tail -1 $O/r05t_first.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/r05t_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05t_suite.log; exit 1; }
tail -1 $O/r05t_suite.log
B="--steps 1 --warmup 0 --c2-items 4096 --tagg-groups 0 --cpu-sample 0 --c5 1 --keys 0 --latency-calls 0 --host-path 0 --rlc-variants i --rlc-steps 3"
timeout -k 10 400 python -u bench.py $B > $O/r05t_c5.json 2> $O/r05t_c5.err || { echo "c5 failed"; tail -20 $O/r05t_c5.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05t_c5.json')); r=d['rlc_batch_verify']['i_root_per_validator']; c=d['full_slot_mix']
print('C4i', r['ms_per_batch'], r['failed_batch_check_ms_per_batch'], r['auto_mode_amortized_ms_per_batch'], 'C5', c['ms_per_slot'], c['failed_batch_check_ms_per_slot'], c['auto_mode_amortized_ms_per_slot'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c5trace3 -o run -- python3 $R/bench.py $B > $O/c5trace3/out.json 2> $O/c5trace3/err.log || { echo "trace failed"; tail -20 $O/c5trace3/err.log; exit 1; }
echo done
