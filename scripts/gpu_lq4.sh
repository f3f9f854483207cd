#!/bin/bash
# Lane quads: the lane-pair/quad parity tests, the fused sigagg test in every layout, the Verify size sweep
# (single / lanes / quads), then the C3 A/B over the given variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lg2.py tests/test_gpu_small_order.py tests/test_gpu_r02.py -x -v --timeout 300 --timeout-method thread -k "lanes or layout or mode or fused or small_order" > gpurun_out/pt_lq4.log 2>&1 || { tail -40 gpurun_out/pt_lq4.log; exit 1; }
tail -3 gpurun_out/pt_lq4.log
timeout -k 10 300 python -u charon_amd/tools/pair_sweep.py > gpurun_out/pair_sweep.txt 2> gpurun_out/pair_sweep.err || { tail -20 gpurun_out/pair_sweep.err; exit 1; }
cat gpurun_out/pair_sweep.txt
bash scripts/gpu_c3_ab.sh "$@"
