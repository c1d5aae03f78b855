#!/bin/bash
# the C2 headline line (with its end-to-end arapOptimization timings) and deformationOptimization
# at C2, after the host graph / upload changes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04e2e}
mkdir -p $OUT
cd $R
DEFTRI_CALL_TIMING=1 DEFTRI_UPLOAD_TIMING=1 timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));r=d['roofline'];print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], d['cpu_baseline']['value'], d['end_to_end_arap_optimization'])"
DEFTRI_CALL_TIMING=1 timeout -k 10 600 python -u bench.py --workload deformation --corr 100000 --no-cpu-baseline > $OUT/bench_def_c2.json 2> $OUT/bench_def_c2.err || { echo def c2 failed; tail -20 $OUT/bench_def_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_def_c2.json'));print('def c2', round(d['value'],2), d['config'])"
