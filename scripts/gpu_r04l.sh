#!/bin/bash
# Round 4: load-balanced MSM buckets (run lanes + fixup), 8-bucket segments, two-step window fold -- the RLC GPU tests,
# then the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_rlcb.py tests/test_gpu_r04.py tests/test_gpu_configs.py tests/test_gpu_multidev.py > $O/r04l_pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/r04l_pytest.log; exit 1; }
tail -3 $O/r04l_pytest.log
timeout -k 10 500 python -u bench.py > $O/r04l_bench.json 2> $O/r04l_bench.err || { echo "bench failed"; tail -30 $O/r04l_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r04l_bench.json'))
print('C2', d['value'], d['roofline']['kernel_avg_ms'], 'lat', d['drop_in_latency']['p50_ms'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregate_kernel_avg_ms'], 'C5', d['full_slot_mix']['ms_per_slot'])
for k,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(k, v['ms_per_batch'], v['batch_checks'], v['kernel_avg_ms'])"
