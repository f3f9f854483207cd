#!/bin/bash
# A/B of compile-time variants on the C3 workload (10,000 x 7-of-10 + aggregate Verify): the in-tree build, then each
# scratch_ab/libhipbls_<v>.so given on the command line (loaded through HIPBLS_LIB).  Each run has its own limit.
set -o pipefail
mkdir -p gpurun_out
ARGS="--c2-items 4096 --rlc-node-validators 0 --c5 0 --keys 0 --cpu-sample 0 --steps 2 --warmup 1 --tagg-steps 6"
timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/c3_base.json 2> gpurun_out/c3_base.err || exit 1
for v in "$@"; do
  HIPBLS_LIB=scratch_ab/libhipbls_$v.so timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/c3_$v.json 2> gpurun_out/c3_$v.err || exit 1
done
for f in gpurun_out/c3_*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['threshold_aggregates_per_s'], d.get('threshold_aggregate_kernel_avg_ms'))" $f
done
