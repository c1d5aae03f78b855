#!/bin/bash
# round 4: kernel-trace gaps of the timed loop with the device-driven LM (DEFTRI_DEVICE_LM=1)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04dlm}
mkdir -p $OUT
cd $R
TAG=${TAG:-r04dlm} bash tools/r04_ab.sh "" "DEFTRI_DEVICE_LM=1"
cd /tmp && export TMPDIR=/tmp
DEFTRI_DEVICE_LM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 1 --no-cpu-baseline --no-e2e --trace-markers > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt && head -24 $OUT/gaps.txt
