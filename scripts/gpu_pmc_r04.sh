#!/bin/bash
# Round-4 PMC passes on HEAD: one rocprofv3 --pmc run per counter group over one step of a
# workload, each under its own time limit.  WL=c2 | c3 | c4 picks the bench arguments; the integer-VALU group is
# built from the counters `rocprofv3 --list-avail` reports on this box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${WL:-c2}
O=$R/gpurun_out/pmc_$WL
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
case $WL in
  c2) ARGS="--steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0";;
  c3) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-steps 1 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0";;
  c4) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-groups 0 --rlc-steps 1 --rlc-variants i,all_valid,ii_all_valid --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0";;
esac
if [ ! -s $R/gpurun_out/counters_avail.txt ]; then
  timeout -s KILL 90 rocprofv3 --list-avail > $R/gpurun_out/counters_avail.txt 2>&1 || true
fi
INT=$(grep -o -E "\bSQ_INSTS_VALU_(INT32|INT64|CVT|TRANS_F32|TRANS_F64|FMA_F32|ADD_F32|MUL_F32)\b" $R/gpurun_out/counters_avail.txt | sort -u | head -6 | tr '\n' ' ')
echo "integer/VALU-type counters: $INT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVES $INT"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/bench.py $ARGS > $O/p$i.out 2> $O/p$i.err || { echo "pmc pass $i failed"; tail -20 $O/p$i.err; exit 1; }
done
python3 $R/scripts/pmc_summary_r04.py $O > $O/summary.json && echo "summary: $O/summary.json"
