#!/bin/bash
# BA workload: GPU tests of the BA path, bench lines (500k x 8 and 50k x 8), rocprofv3 kernel stats.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ba_bench}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_ba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_ba.log 2>&1 || { tail -40 $OUT/pytest_ba.log; exit 1; }
tail -2 $OUT/pytest_ba.log
timeout -k 10 600 python3 bench.py --workload ba --ba-points 500000 --steps 10 --warmup 2 > $OUT/bench_ba500k.json 2> $OUT/bench_ba500k.err || { tail -30 $OUT/bench_ba500k.err; exit 1; }
cat $OUT/bench_ba500k.json
timeout -k 10 600 python3 bench.py --workload ba --ba-points 50000 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_ba50k.json 2> $OUT/bench_ba50k.err || { tail -30 $OUT/bench_ba50k.err; exit 1; }
cat $OUT/bench_ba50k.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --workload ba --ba-points 500000 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_ba_prof.json 2> $OUT/bench_ba_prof.err
ls $OUT/prof
