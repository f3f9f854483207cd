#!/bin/bash
# Quick GPU check after a kernel change: op microbenchmark, the -m gpu suite, a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./charon_amd/tools/op_probe > gpurun_out/op_probe.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/op_probe.txt; tail -3 gpurun_out/pytest_gpu.log
exit $rc
