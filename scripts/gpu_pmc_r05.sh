#!/bin/bash
# Round-5 PMC passes (one rocprofv3 --pmc run per counter group, each under its own time limit).  WL=lat: the n = 1
# drop-in latency loop (40 queued single Verifies, run with HIPBLS_LAT_REPLICAS=1 so the counters are one copy's; the C2 step runs 8,192 items so it takes quads and the octet
# kernels k_verify_prep8 / k_verify_pair_lq8 are the latency loop's alone).  WL=c2 | c3 | c4 as in round 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
WL=${WL:-lat}
O=$R/gpurun_out/pmc5_$WL
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
case $WL in
  lat) ARGS="--c2-items 8192 --steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 40";;
  c2) ARGS="--steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0";;
  c3) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-steps 1 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0";;
  c4) ARGS="--c2-items 40960 --steps 1 --warmup 0 --tagg-groups 0 --rlc-steps 1 --rlc-variants i,all_valid,ii_all_valid --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0";;
esac
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 $R/bench.py $ARGS > $O/p$i.out 2> $O/p$i.err || { echo "pmc pass $i failed"; tail -20 $O/p$i.err; exit 1; }
done
python3 $R/scripts/pmc_summary_r04.py $O > $O/summary.json && echo "summary: $O/summary.json"
