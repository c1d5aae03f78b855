#!/bin/bash
# One GPU session: parity tests, smoke, bench (CPU baseline + end-to-end), rocprofv3 kernel stats,
# the PCG product's HBM counters, the 500k two-view bench.  Every GPU step has its own time limit;
# steps are chained so the first failure ends the session.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r02}
mkdir -p $OUT $OUT/pmc
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 600 python3 bench.py --corr 500000 --no-cpu-baseline --no-e2e > $OUT/bench_500k.json 2> $OUT/bench_500k.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/bench_prof.json 2> $OUT/bench_prof.err
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc/fetch -o run -- python3 $B > $OUT/pmc/fetch.json 2> $OUT/pmc/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc/write -o run -- python3 $B > $OUT/pmc/write.json 2> $OUT/pmc/write.err
find $OUT/prof -name "*kernel_stats.csv" | head -5
