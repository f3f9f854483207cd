#!/bin/bash
# A/B of compile-time variants on the C2 workload (65,536 individual Verify): the in-tree build, then each
# scratch_ab/libhipbls_<v>.so given on the command line (loaded through HIPBLS_LIB).  Each run has its own limit.
set -o pipefail
mkdir -p gpurun_out
ARGS="--rlc-node-validators 0 --c5 0 --keys 0 --cpu-sample 0 --steps 5 --warmup 1 --tagg-groups 1000 --tagg-steps 1"
timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/c2_base.json 2> gpurun_out/c2_base.err || exit 1
for v in "$@"; do
  HIPBLS_LIB=scratch_ab/libhipbls_$v.so timeout -k 10 240 python -u bench.py $ARGS > gpurun_out/c2_$v.json 2> gpurun_out/c2_$v.err || exit 1
done
for f in gpurun_out/c2_*.json; do
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])" $f
done
