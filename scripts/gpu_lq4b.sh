#!/bin/bash
# Quad final exponentiation: its GPU unit tests, the layout/parity tests, the Verify size sweep, the C3 A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_lg2.py tests/test_gpu_small_order.py tests/test_gpu_r02.py -x -v --timeout 300 --timeout-method thread -k "quad or lanes or layout or mode or fused or small_order or exp" > gpurun_out/pt_lq4b.log 2>&1 || { tail -40 gpurun_out/pt_lq4b.log; exit 1; }
tail -3 gpurun_out/pt_lq4b.log
timeout -k 10 300 python -u charon_amd/tools/pair_sweep.py 1,1024,10000,16384 > gpurun_out/pair_sweep.txt 2> gpurun_out/pair_sweep.err || { tail -20 gpurun_out/pair_sweep.err; exit 1; }
cat gpurun_out/pair_sweep.txt
bash scripts/gpu_c3_ab.sh "$@"
