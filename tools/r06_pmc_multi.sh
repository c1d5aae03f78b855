#!/bin/bash
# round 6: FETCH_SIZE / WRITE_SIZE of the multi-pair tile kernels (C3, C5), one rocprofv3 pass per
# counter (kernel trace only), each under its own time limit; summarized on the CPU afterwards
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06pmcm}
cd /tmp && export TMPDIR=/tmp
for w in ${WLS:-c3 c5}; do
  OUT=$R/gpurun_out/$TAG/$w
  mkdir -p $OUT
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo "$w fetch failed"; tail -5 $OUT/pmc_fetch.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo "$w write failed"; tail -5 $OUT/pmc_write.err; exit 1; }
  echo "$w ok"
done
