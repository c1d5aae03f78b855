#!/bin/bash
# C4 host side on the box: graph build and iterative-plan stage times (DEFTRI_GRAPH_TIMING,
# DEFTRI_PLAN_TIMING) around a short C4 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04c4h}
mkdir -p $OUT
cd $R
DEFTRI_GRAPH_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_UPLOAD_TIMING=1 timeout -k 10 600 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo c4 failed; tail -20 $OUT/bench_c4.err; exit 1; }
grep -v "pair [0-9]*:" $OUT/bench_c4.err | tail -30
