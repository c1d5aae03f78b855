#!/bin/bash
# round 3: C2 A/B of the CG chain variants (merged 2 launches / merged + alpha kernel / three-launch), alternating
set -o pipefail
OUT=gpurun_out/r03ab3
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for v in m k t m2 k2 t2; do
  case $v in m*) E="";; k*) E="DEFTRI_SP_ALPHA_KERNEL=1";; t*) E="DEFTRI_SP_NO_MERGE=1";; esac
  env $E timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/ab_$v.json 2> $OUT/ab_$v.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/ab_$v.json').read().strip().splitlines()[-1]);c=d['config'];print('$v', '$E', round(d['value'],1), c['ms_per_cg_iteration_profiled'], d['roofline']['frac'], c.get('cg_iterations_per_trial'), c.get('trials_per_iteration'))"
done
