#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in the same pass).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err
ls $OUT/prof
