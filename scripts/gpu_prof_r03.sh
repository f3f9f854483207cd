#!/bin/bash
# Round-3 profiles on HEAD: PMC passes over one C2 verify step (scripts/gpu_pmc.sh) summarized for k_verify_fused,
# then a kernel-trace + stats run of the default bench (every config).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_pmc.sh || exit 1
python3 $R/scripts/pmc_summary.py $R/gpurun_out/pmc k_verify_fused $R/gpurun_out/r03_pmc_verify.json \
  "rocprofv3 --pmc, 4 separate passes over one C2 step (65,536 verifies), round-3 build" > /dev/null || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-sample 0 > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof_bench.err || { echo "trace failed"; tail -20 $R/gpurun_out/prof_bench.err; exit 1; }
find $R/gpurun_out/prof -name '*stats*'
cat $R/gpurun_out/r03_pmc_verify.json
