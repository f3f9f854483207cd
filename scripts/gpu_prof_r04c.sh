#!/bin/bash
# Round 4, profiles C: kernel traces of (1) the C4 variants with the G1 MSM per committee root and (2) the n = 1 drop-in
# latency calls (verify_prep + the pairing check per call), each with its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04c_c4 -o c4 -- python3 $R/bench.py --c2-items 40960 --steps 1 --warmup 0 --tagg-groups 0 --rlc-steps 2 --c5 0 --keys 0 --latency-calls 0 --cpu-sample 0 > $O/prof_r04c_c4.json 2> $O/prof_r04c_c4.err || { echo "c4 trace failed"; tail -20 $O/prof_r04c_c4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r04c_lat -o lat -- python3 $R/bench.py --c2-items 4096 --steps 1 --warmup 0 --tagg-groups 0 --rlc-node-validators 0 --c5 0 --keys 0 --latency-calls 100 --cpu-sample 0 > $O/prof_r04c_lat.json 2> $O/prof_r04c_lat.err || { echo "latency trace failed"; tail -20 $O/prof_r04c_lat.err; exit 1; }
find $O/prof_r04c_c4 $O/prof_r04c_lat -name '*stats*'
