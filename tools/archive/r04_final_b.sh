#!/bin/bash
# round 4 final measurements, part B: the multi-keyframe workloads at Simulation.yaml's 25 LM
# iterations, and deformationOptimization end to end at C1 (CPU leg) and C2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04f}
mkdir -p $OUT
cd $R
for w in c3 c5 c4; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 25 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo $w failed; tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));r=d['roofline'];print('$w', round(d['value'],2), round(d['ms_per_step'],2), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], (d['cpu_baseline'] or {}).get('value'))"
done
timeout -k 10 600 python -u bench.py --workload deformation --corr 1000 > $OUT/bench_def_c1.json 2> $OUT/bench_def_c1.err || { echo def c1 failed; tail -20 $OUT/bench_def_c1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_def_c1.json'));print('def C1', round(d['value'],2), d['config'], (d['cpu_baseline'] or {}).get('value'))"
