#!/bin/bash
# PMC passes for one workload (round 6; the round-4/5 runners folded into one): one rocprofv3 --pmc run per counter
# group, each under its own time limit, then scripts/pmc_summary_r04.py folds them into <out>/summary.json
# (scripts/pmc_commit_r04.py <rev> <round> <prefix> writes profiles/<round>/pmc_<wl>.json from it).
#   WL=c2 | c3 | c4 | lat   PREFIX (default pmc6_) -> gpurun_out/<PREFIX><WL>/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${WL:-c2}
O=$R/gpurun_out/${PREFIX:-pmc6_}$WL
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
case $WL in
  lat) ARGS="--c2-items 8192 --steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --host-path 0 --latency-calls 40";;
  c2) ARGS="--steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --host-path 0 --latency-calls 0";;
  c3) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-steps 1 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --host-path 0 --latency-calls 0";;
  c4) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-groups 0 --rlc-steps 1 --rlc-variants i,all_valid,ii_all_valid --c5 0 --keys 0 --host-path 0 --latency-calls 0 --cpu-sample 0";;
  *) echo "unknown WL $WL"; exit 2;;
esac
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$O/p$i" -o run -- python3 "$R/bench.py" $ARGS \
    > "$O/p$i.out" 2> "$O/p$i.err" || { echo "pmc pass $i failed"; tail -20 "$O/p$i.err"; exit 1; }
done
python3 "$R/scripts/pmc_summary_r04.py" "$O" > "$O/summary.json" && echo "summary: $O/summary.json"
