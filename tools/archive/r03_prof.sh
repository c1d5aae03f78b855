#!/bin/bash
# round-3 measurement pass on the default (iterative) plan at C2: the headline bench line (CPU
# baseline + end-to-end), a rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE in separate passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r03h}
mkdir -p $OUT
cd $R && timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('C2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['cpu_baseline']['value'], d['end_to_end_arap_optimization'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo fetch failed; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo write failed; tail -5 $OUT/pmc_write.err; exit 1; }
ls $OUT/prof $OUT/fetch
