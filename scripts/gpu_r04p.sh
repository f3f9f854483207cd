#!/bin/bash
# Round 4, end: PMC passes over the C3 workload at the merged sigagg kernels, then the two-rank bench rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
rm -rf gpurun_out/pmc_c3
WL=c3 bash scripts/gpu_pmc_r04.sh > gpurun_out/pmc_c3.log 2>&1 || { echo "pmc c3 failed"; tail -20 gpurun_out/pmc_c3.log; exit 1; }
tail -1 gpurun_out/pmc_c3.log
bash scripts/gpu_bench_rehearse.sh > gpurun_out/rehearse_r04p.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/rehearse_r04p.log; exit 1; }
tail -2 gpurun_out/rehearse_r04p.log | cut -c1-400
