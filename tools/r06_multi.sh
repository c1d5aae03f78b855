#!/bin/bash
# round 6: the multi-keyframe workloads (BASELINE C3-C5) on the multi-pair tile chain, one MI355X
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06multi}
STEPS=${2:-25}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for w in c3 c5 c4; do
  timeout -k 10 500 python -u bench.py --workload $w --steps $STEPS --warmup 1 --no-cpu-baseline > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "$w failed"; tail -5 $OUT/bench_$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$w.json')); r=d.get('roofline',{}); c=d['config']
print('$w', round(d['value'],3), round(d['ms_per_step'],2), r.get('frac_survey'), r.get('cg_iteration_us'), r.get('tiles'), c.get('cg_iterations_per_pcg_trial'), c.get('trials_per_iteration'))"
done
