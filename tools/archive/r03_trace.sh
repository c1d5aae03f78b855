#!/bin/bash
# round 3: kernel trace of the timed C2 loop (window between bench.py's trace markers) + stats
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e --trace-markers > $R/$OUT/prof.json 2> $R/$OUT/prof.err || { echo trace failed; tail -5 $R/$OUT/prof.err; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt
