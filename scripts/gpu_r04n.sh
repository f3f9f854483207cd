#!/bin/bash
# Round 4, end: the RLC GPU tests and the default bench on the final MSM build, then the PMC passes (C2, C3, C4) at
# this commit for the committed counters (scripts/pmc_commit_r04.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_r04l.sh || exit 1
for wl in c2 c3 c4; do
  WL=$wl bash scripts/gpu_pmc_r04.sh > gpurun_out/pmc_$wl.log 2>&1 || { echo "pmc $wl failed"; tail -20 gpurun_out/pmc_$wl.log; exit 1; }
  tail -1 gpurun_out/pmc_$wl.log
done
