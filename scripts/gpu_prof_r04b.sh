#!/bin/bash
# Round-4 profiles, part B: PMC passes over the C4 stages, then a kernel trace + stats of the default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=c4 bash $R/scripts/gpu_pmc_r04.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r04 -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 --latency-calls 0 > $R/gpurun_out/prof_r04_bench.json 2> $R/gpurun_out/prof_r04_bench.err || { echo "trace failed"; tail -20 $R/gpurun_out/prof_r04_bench.err; exit 1; }
find $R/gpurun_out/prof_r04 -name '*stats*'
