#!/bin/bash
# Round 5: (1) the whole GPU suite on the product build (replica race with 64-byte-aligned race words; RLC tail pairs
# off), then the default bench; (2) the lazy-reduction A/B: C2 on the product build and on
# charon_amd/libhipbls_lazy.so (-DBLS_LAZY_FP6=1), alternating, then the PMC groups of k_verify_fused on both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
if [ "${1:-suite}" = suite ]; then
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/r05c_suite.log 2>&1 || { echo "suite failed"; tail -40 $O/r05c_suite.log; exit 1; }
tail -1 $O/r05c_suite.log
timeout -k 10 500 python -u bench.py > $O/r05c_bench.json 2> $O/r05c_bench.err || { echo "bench failed"; tail -30 $O/r05c_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/r05c_bench.json'))
print('C2', d['value'], d['roofline']['frac'], 'C3', d['threshold_aggregates_per_s'], d['threshold_aggregates_per_s_two_streams'], 'C5', d['full_slot_mix']['ms_per_slot'])
print('lat', d['drop_in_latency'])
print('host', d['host_path'])
for kk,v in d['rlc_batch_verify'].items():
    if isinstance(v,dict): print(kk, v.get('ms_per_batch'))"
exit 0
fi
C2="--steps 5 --warmup 1 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $C2 > $O/r05c_c2_prod$k.json 2> $O/r05c_c2_prod$k.err || { echo "c2 prod failed"; tail -20 $O/r05c_c2_prod$k.err; exit 1; }
  HIPBLS_LIB=$R/charon_amd/libhipbls_lazy.so timeout -k 10 300 python -u bench.py $C2 > $O/r05c_c2_lazy$k.json 2> $O/r05c_c2_lazy$k.err || { echo "c2 lazy failed"; tail -20 $O/r05c_c2_lazy$k.err; exit 1; }
done
for f in $O/r05c_c2_prod1.json $O/r05c_c2_lazy1.json $O/r05c_c2_prod2.json $O/r05c_c2_lazy2.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0"
for v in prod lazy; do
  LIBV=""; [ $v = lazy ] && LIBV=$R/charon_amd/libhipbls_lazy.so
  i=0; mkdir -p $O/pmc5_lazy_$v
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE GRBM_COUNT" \
             "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64"; do
    i=$((i+1))
    HIPBLS_LIB=$LIBV timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc5_lazy_$v/p$i -o run -- python3 $R/bench.py $ARGS > $O/pmc5_lazy_$v/p$i.out 2> $O/pmc5_lazy_$v/p$i.err || { echo "pmc $v pass $i failed"; tail -5 $O/pmc5_lazy_$v/p$i.err; exit 1; }
  done
  python3 $R/scripts/pmc_summary_r04.py $O/pmc5_lazy_$v > $O/pmc5_lazy_$v/summary.json
done
python3 -c "
import json
for v in ('prod','lazy'):
    d=json.load(open('$O/pmc5_lazy_'+v+'/summary.json'))
    k=[x for x in d if x.endswith('k_verify_fused')][0]; e=d[k]
    print(v, {x: e.get(x) for x in ('valu_insts_per_wave','sq_insts_valu_int64_per_wave','valu_util','wait_any_frac','hbm_bytes_per_launch_raw','duration_ms_profiled')})"
