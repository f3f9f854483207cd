#!/bin/bash
# Round 4: inlined additions in the scalar multiplications -- the affected GPU tests, then the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_units.py tests/test_gpu_r02.py tests/test_gpu_rlcb.py tests/test_gpu_lg2.py tests/test_gpu_parity.py tests/test_gpu_small_order.py tests/test_gpu_rlc.py > $O/r04i_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04i_pytest.log; exit 1; }
tail -3 $O/r04i_pytest.log
timeout -k 10 500 python -u bench.py > $O/r04i_bench.json 2> $O/r04i_bench.err || { echo "bench failed"; tail -30 $O/r04i_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04i_bench.json'))
print('C2', d['value'], d['roofline']['kernel_avg_ms'], 'lat', d['drop_in_latency']['p50_ms'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregate_kernel_avg_ms'], 'C5', d['full_slot_mix']['ms_per_slot'])
for k,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(k, v['ms_per_batch'], v['kernel_avg_ms'])"
