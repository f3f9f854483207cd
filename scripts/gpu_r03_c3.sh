#!/bin/bash
# Round 3: the -m gpu suite on the in-tree build, then the C3 A/B (scripts/gpu_c3_ab.sh) over the given variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash scripts/gpu_c3_ab.sh "$@"
