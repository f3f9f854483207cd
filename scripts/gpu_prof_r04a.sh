#!/bin/bash
# Round-4 profiles, part A: PMC passes over one C2 step and one C3 step on HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=c2 bash $R/scripts/gpu_pmc_r04.sh && WL=c3 bash $R/scripts/gpu_pmc_r04.sh
cd $R && timeout -k 10 300 python -u bench.py --rlc-node-validators 0 --c5 0 > $R/gpurun_out/r04_bench_quick.json 2> $R/gpurun_out/r04_bench_quick.err || { echo "bench failed"; tail -20 $R/gpurun_out/r04_bench_quick.err; exit 1; }
cat $R/gpurun_out/r04_bench_quick.json
