#!/bin/bash
# Round 5: (1) the RLC tail sub-batch's fallback on lane pairs (HIPBLS_RLC_TAIL_PAIRS=1): the RLC/config GPU tests with
# it on, then C4(i) with it off/on alternating; (2) the lazy-reduction PMC pair: k_verify_fused
# counters on the product build and on charon_amd/libhipbls_lazy.so.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
export PYTHONPATH=$R
HIPBLS_RLC_TAIL_PAIRS=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_rlc.py tests/test_gpu_rlcb.py > $O/r05f_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/r05f_tests.log; exit 1; }
tail -1 $O/r05f_tests.log
C4="--steps 1 --warmup 0 --tagg-groups 0 --cpu-sample 0 --c5 0 --keys 0 --latency-calls 0 --host-path 0 --c2-items 4096 --rlc-variants i --rlc-steps 3"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py $C4 > $O/r05f_c4_off$k.json 2> $O/r05f_c4_off$k.err || { echo "c4 off failed"; tail -20 $O/r05f_c4_off$k.err; exit 1; }
  HIPBLS_RLC_TAIL_PAIRS=1 timeout -k 10 300 python -u bench.py $C4 > $O/r05f_c4_on$k.json 2> $O/r05f_c4_on$k.err || { echo "c4 on failed"; tail -20 $O/r05f_c4_on$k.err; exit 1; }
  for f in $O/r05f_c4_off$k.json $O/r05f_c4_on$k.json; do python3 -c "
import json; d=json.load(open('$f'))['rlc_batch_verify']['i_root_per_validator']; print('$f'.split('/')[-1], d['ms_per_batch'], d['items_fallback'], d['kernel_avg_ms'])"; done
done
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
    print(v, {x: e.get(x) for x in ('valu_insts_per_wave','sq_insts_valu_int64_per_wave','valu_util','wait_any_frac','hbm_bytes_per_launch_raw','duration_ms_profiled')}, e['counters_per_launch'].get('_scratch_B'))"
