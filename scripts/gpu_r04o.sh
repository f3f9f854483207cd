#!/bin/bash
# Round 4: sigagg as three kernels on the caller's stream with two workspace sets and chained phase A -- the sigagg
# GPU tests (incl. four calls in flight on two streams), then the default bench (C3 single- and two-stream).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_r04.py tests/test_gpu_r02.py tests/test_gpu_multidev.py tests/test_gpu_small_order.py tests/test_gpu_lg2.py > $O/r04o_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04o_pytest.log; exit 1; }
tail -3 $O/r04o_pytest.log
timeout -k 10 500 python -u bench.py > $O/r04o_bench.json 2> $O/r04o_bench.err || { echo "bench failed"; tail -30 $O/r04o_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04o_bench.json'))
print('C2', d['value'], 'lat', d['drop_in_latency']['p50_ms'], 'C3', d['threshold_aggregates_per_s'], 'C3x2', d['threshold_aggregates_per_s_two_streams'], d['threshold_aggregate_kernel_avg_ms'], d['threshold_aggregate_roofline'], 'C5', d['full_slot_mix']['ms_per_slot'])"
