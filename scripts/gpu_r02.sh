#!/bin/bash
# Round-2 GPU check: full -m gpu suite, then a short bench.  Each GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
