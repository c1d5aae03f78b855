#!/bin/bash
# Full GPU test suite, BA bench lines + rocprof, C2 bench line, per-level factor profile.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-mix}
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python3 bench.py --workload ba --ba-points 500000 --steps 10 --warmup 2 > $OUT/bench_ba500k.json 2> $OUT/bench_ba500k.err || { tail -30 $OUT/bench_ba500k.err; exit 1; }
cat $OUT/bench_ba500k.json
timeout -k 10 600 python3 bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python3 tools/prof_levels.py > $OUT/prof_levels.txt 2>&1 || { tail -30 $OUT/prof_levels.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ba -o run -- python3 $R/bench.py --workload ba --ba-points 500000 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_ba_prof.json 2> $OUT/bench_ba_prof.err
ls $OUT/prof_ba
