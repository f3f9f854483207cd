#!/bin/bash
# Round-2 profiles on HEAD: PMC passes over one C2 verify step (scripts/gpu_pmc.sh), then a kernel-trace + stats run
# of the default bench (every config) whose summary goes to profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_pmc.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo "trace failed"; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
find $R/gpurun_out/prof -name '*stats*'
