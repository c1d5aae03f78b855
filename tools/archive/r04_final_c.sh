#!/bin/bash
# round 4 final measurements, part C: the 500k-correspondence two-view line (north-star size) with
# its CPU baseline, and deformationOptimization at C2 (device only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04f}
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u bench.py --corr 500000 --no-e2e > $OUT/bench_500k.json 2> $OUT/bench_500k.err || { echo 500k failed; tail -20 $OUT/bench_500k.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_500k.json'));r=d['roofline'];print('500k', round(d['value'],2), round(d['ms_per_step'],3), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], d['cpu_baseline'])"
