#!/bin/bash
# Two-rank rehearsal of the multi-GPU bench path on a one-GPU box: both ranks share cuda:0, the collectives run over
# gloo through host memory (HIPBLS_BENCH_BACKEND=gloo); checks slicing, the gathered node bitmaps and aggregates.
set -o pipefail
mkdir -p gpurun_out
HIPBLS_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --c2-items 8192 --tagg-groups 1000 \
  --tagg-steps 1 --rlc-node-validators 16384 --rlc-steps 1 --cpu-sample 0 > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err
rc=$?
tail -5 gpurun_out/rehearse.err; cat gpurun_out/rehearse.json
exit $rc
