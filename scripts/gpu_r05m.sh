#!/bin/bash
# Round 5: one shared Miller accumulator for lq4_verify's two pairs (BLS_LQ4_SHARED, product build) against the split
# loops (charon_amd/libhipbls_split.so, -DBLS_LQ4_SHARED=0): parity tests, the whole suite, then the n = 1 race trace
# and C3 on both builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/rt_shared $O/rt_split
cd $R
export PYTHONPATH=$R
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_lg2.py tests/test_gpu_small_order.py tests/test_gpu_r04.py tests/test_gpu_r05.py tests/test_gpu_units.py > $O/r05m_first.log 2>&1 || { echo "first tests failed"; tail -40 $O/r05m_first.log; exit 1; }
tail -1 $O/r05m_first.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/r05m_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05m_suite.log; exit 1; }
tail -1 $O/r05m_suite.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rt_shared -o run -- python3 -u scripts/race_trace.py 100 8,8,1 > $O/rt_shared/host.jsonl 2> $O/rt_shared/err.log || { echo "race trace shared failed"; tail -20 $O/rt_shared/err.log; exit 1; }
HIPBLS_LIB=$R/charon_amd/libhipbls_split.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rt_split -o run -- python3 -u scripts/race_trace.py 100 8,8,1 > $O/rt_split/host.jsonl 2> $O/rt_split/err.log || { echo "race trace split failed"; tail -20 $O/rt_split/err.log; exit 1; }
C3="--steps 1 --warmup 0 --c2-items 4096 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0 --tagg-steps 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $C3 > $O/r05m_c3_shared$k.json 2> $O/r05m_c3_shared$k.err || { echo "c3 shared failed"; tail -20 $O/r05m_c3_shared$k.err; exit 1; }
  HIPBLS_LIB=$R/charon_amd/libhipbls_split.so timeout -k 10 300 python -u bench.py $C3 > $O/r05m_c3_split$k.json 2> $O/r05m_c3_split$k.err || { echo "c3 split failed"; tail -20 $O/r05m_c3_split$k.err; exit 1; }
  for f in $O/r05m_c3_shared$k.json $O/r05m_c3_split$k.json; do python3 -c "
import json; d=json.load(open('$f')); print('$f'.split('/')[-1], d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], d.get('threshold_aggregate_kernel_ms'))"; done
done
