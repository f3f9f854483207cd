#!/bin/bash
# Lane-pair pairing checks: parity tests, then the Verify size sweep (single vs pair layouts), then a short bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_lg2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pt_lg2.log 2>&1 && \
timeout -k 10 300 python -u charon_amd/tools/pair_sweep.py > gpurun_out/pair_sweep.txt 2> gpurun_out/pair_sweep.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-sample 0 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/pt_lg2.log; cat gpurun_out/pair_sweep.txt; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/bench.json
exit $rc
