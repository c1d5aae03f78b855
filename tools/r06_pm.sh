#!/bin/bash
# round 6: multi-pair tiles with each pair's units in the Morton order of that pair's own mesh positions
# (DEFTRI_TILE_PAIR_MORTON=1) against the global group order: C3, C5 (and C4) on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06pm}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for w in ${WLS:-c3 c5}; do
for v in 0 1; do
  if [ $v = 1 ]; then export DEFTRI_ROWS_KF_MORTON=1; else unset DEFTRI_ROWS_KF_MORTON; fi
  timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/${w}_$v.json 2> $OUT/${w}_$v.err || { echo "$w failed"; tail -5 $OUT/${w}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/${w}_$v.json')); r=d['roofline']; c=d['config']; t=d['trial_kernel_ms']
print('$w', 'pm=$v', round(d['value'],3), r['tiles'], r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'], r['frac_survey'], c['cg_iterations_per_pcg_trial'], t.get('sp_glin_rows'), c['chi2_final'])"
done
done
