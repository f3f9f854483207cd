#!/bin/bash
# One parameterised GPU runner (round 6: replaces the per-run scripts/gpu_r0*.sh).  Each argument is a step, run in
# order under its own time limit; the first failing step ends the call (no retries):
#
#   suite                 the whole GPU test suite                         -> gpurun_out/<tag>_suite.log
#   smoke                 __graft_entry__.smoke()                          -> gpurun_out/<tag>_smoke.log
#   bench                 the default bench line                           -> gpurun_out/<tag>_bench.json
#   prof                  the default bench under rocprofv3 --kernel-trace --stats -> gpurun_out/<tag>_prof/
#   rlc:<lib>:<name>      the C4(i) + C5 part of the bench with HIPBLS_LIB=<lib> (A/B of compile-time variants)
#   c2:<lib>:<name>       the C2 part of the bench alone (5 steps) with HIPBLS_LIB=<lib>; repeat the step to alternate
#   c3:<lib>:<name>       the C3 part (sigagg, 6 timed calls) with a 4,096-item C2, HIPBLS_LIB=<lib>
#   pmc:<counters>:<name> one rocprofv3 --pmc pass over a short C2-only bench -> gpurun_out/<tag>_pmc_<name>/
#   pmcset:<wl>           the five counter passes of scripts/gpu_pmc.sh for workload c2|c3|c4|lat -> gpurun_out/pmc6_<wl>/
#   ceiling[:<bin>:<name>] charon_amd/tools/ceiling_probe or <bin> (the product routines alone, every SIMD) -> <tag>_ceiling[_<name>].txt
#   py:<file>             python -u <file> (a probe script)                -> gpurun_out/<tag>_<basename>.log
#
# TAG (environment, default "run") prefixes every output.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
T=${TAG:-run}
mkdir -p "$O"
cd "$R" || exit 1
export TMPDIR=/tmp
RLC_ARGS="--steps 2 --warmup 1 --tagg-groups 0 --latency-calls 0 --host-path 0 --keys 0 --cpu-sample 0 --rlc-steps 3 --rlc-variants i"
C2_ONLY="--tagg-groups 0 --latency-calls 0 --host-path 0 --keys 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0"
C3_ONLY="--c2-items 4096 --steps 2 --warmup 1 --tagg-steps 6 --latency-calls 0 --host-path 0 --keys 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0"
C2_ARGS="--steps 3 --warmup 1 --tagg-groups 0 --latency-calls 0 --host-path 0 --keys 0 --cpu-sample 0 --rlc-node-validators 0 --c5 0"

for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    suite)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
        > "$O/${T}_suite.log" 2>&1 || { echo "suite failed"; tail -40 "$O/${T}_suite.log"; exit 1; }
      tail -1 "$O/${T}_suite.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/${T}_smoke.log" 2>&1 \
        || { echo "smoke failed"; tail -20 "$O/${T}_smoke.log"; exit 1; }
      tail -1 "$O/${T}_smoke.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$O/${T}_bench.json" 2> "$O/${T}_bench.err" \
        || { echo "bench failed"; tail -30 "$O/${T}_bench.err"; exit 1; }
      python3 scripts/bench_summary.py "$O/${T}_bench.json" ;;
    prof)
      mkdir -p "$O/${T}_prof"
      (cd /tmp && timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/${T}_prof" -o run \
        -- python3 -u "$R/bench.py" > "$O/${T}_prof_bench.json" 2> "$O/${T}_prof_bench.err") \
        || { echo "profiled bench failed"; tail -30 "$O/${T}_prof_bench.err"; exit 1; }
      python3 scripts/bench_summary.py "$O/${T}_prof_bench.json" ;;
    rlc:*)
      IFS=: read -r _ lib name <<< "$step"
      HIPBLS_LIB="$R/$lib" timeout -k 10 600 python -u bench.py $RLC_ARGS > "$O/${T}_rlc_${name}.json" \
        2> "$O/${T}_rlc_${name}.err" || { echo "rlc bench failed"; tail -30 "$O/${T}_rlc_${name}.err"; exit 1; }
      python3 scripts/bench_summary.py "$O/${T}_rlc_${name}.json" ;;
    c3:*)
      IFS=: read -r _ lib name <<< "$step"
      k=0
      while [ -e "$O/${T}_c3_${name}_$k.json" ]; do k=$((k+1)); done
      HIPBLS_LIB="$R/$lib" timeout -k 10 300 python -u bench.py $C3_ONLY > "$O/${T}_c3_${name}_$k.json" \
        2> "$O/${T}_c3_${name}_$k.err" || { echo "c3 bench failed"; tail -30 "$O/${T}_c3_${name}_$k.err"; exit 1; }
      python3 scripts/bench_summary.py "$O/${T}_c3_${name}_$k.json" ;;
    c2:*)
      IFS=: read -r _ lib name <<< "$step"
      k=0
      while [ -e "$O/${T}_c2_${name}_$k.json" ]; do k=$((k+1)); done
      HIPBLS_LIB="$R/$lib" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 $C2_ONLY > "$O/${T}_c2_${name}_$k.json" \
        2> "$O/${T}_c2_${name}_$k.err" || { echo "c2 bench failed"; tail -30 "$O/${T}_c2_${name}_$k.err"; exit 1; }
      python3 scripts/bench_summary.py "$O/${T}_c2_${name}_$k.json" ;;
    pmc:*)
      IFS=: read -r _ counters name <<< "$step"
      mkdir -p "$O/${T}_pmc_${name}"
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${counters//,/ } --output-format csv \
        -d "$O/${T}_pmc_${name}" -o run -- python3 -u "$R/bench.py" $C2_ARGS \
        > "$O/${T}_pmc_${name}.json" 2> "$O/${T}_pmc_${name}.err") \
        || { echo "pmc pass failed"; tail -20 "$O/${T}_pmc_${name}.err"; exit 1; } ;;
    pmcset:*)
      WL=${step#pmcset:} bash scripts/gpu_pmc.sh > "$O/${T}_pmcset_${step#pmcset:}.log" 2>&1 \
        || { echo "pmc set failed"; tail -20 "$O/${T}_pmcset_${step#pmcset:}.log"; exit 1; }
      tail -1 "$O/${T}_pmcset_${step#pmcset:}.log" ;;
    ceiling|ceiling:*)
      IFS=: read -r _ bin name <<< "$step"
      bin=${bin:-charon_amd/tools/ceiling_probe}
      f="$O/${T}_ceiling${name:+_$name}.txt"
      timeout -k 10 300 "$R/$bin" > "$f" 2>&1 || { echo "ceiling probe failed"; tail -20 "$f"; exit 1; }
      cat "$f" ;;
    py:*)
      f=${step#py:}
      timeout -k 10 600 python -u "$f" > "$O/${T}_$(basename "$f" .py).log" 2>&1 \
        || { echo "$f failed"; tail -30 "$O/${T}_$(basename "$f" .py).log"; exit 1; }
      tail -5 "$O/${T}_$(basename "$f" .py).log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
