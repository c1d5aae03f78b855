#!/bin/bash
# round 4 measurement pass: the headline C2 line (CPU baseline + end-to-end), its rocprofv3 kernel
# stats, the multi-keyframe workloads at Simulation.yaml's 25 iterations, the deformation leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04m}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));r=d['roofline'];print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], d['cpu_baseline']['value'], d['end_to_end_arap_optimization'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
cd $R
for w in c3 c5 c4; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 25 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo $w failed; tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));r=d['roofline'];print('$w', round(d['value'],2), round(d['ms_per_step'],2), r['frac_survey'], r['frac_design'], r['cg_iteration_us'], (d['cpu_baseline'] or {}).get('value'))"
done
