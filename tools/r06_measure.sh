#!/bin/bash
# round 6 measurement pass: the C2 headline line (CPU baseline, end-to-end, 500k and Realcolon legs),
# its rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes of the CG kernels (separate runs,
# kernel trace only), the PMC summary keyed by the plan's algorithmic bytes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06m}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));r=d['roofline'];print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-legs > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-legs > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo fetch failed; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-legs > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo write failed; tail -5 $OUT/pmc_write.err; exit 1; }
cd $R && python3 tools/pmc_sp_summary.py gpurun_out/$TAG gpurun_out/$TAG/pmc_sp_product.json > /dev/null && echo pmc ok
