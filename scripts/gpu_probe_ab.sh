#!/bin/bash
# op-probe variants (paths given as arguments, each under its own time limit), then the A/B bench + -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
i=0
for p in "$@"; do
  i=$((i+1))
  timeout -k 10 150 "$p" > gpurun_out/op$i.txt 2>&1 || { echo "probe $p failed"; exit 1; }
done
bash scripts/gpu_ab.sh
