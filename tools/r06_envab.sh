#!/bin/bash
# round 6: one environment switch (NAME=VAL in $SW) against the default on the working tree: C2 and
# 500k x 2 on tools/tile_ab.py (LM run, profiled trial's CG kernels), C3 / C5 on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06envab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for n in ${NS:-100000 500000}; do
  timeout -k 10 400 python -u tools/tile_ab.py $n 10 - $SW - $SW > $OUT/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -5 $OUT/ab_$n.log; exit 1; }
  python3 -c "
import json
for l in open('$OUT/ab_$n.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print($n, d['env'], d['tiles'], d['cg_us'], d['cg_iteration_us'], d['lm_it_s'], d['trials'][:5], d['pcg_its'])
    elif l.startswith('{\"same'): print(l.strip())
"
done
for w in ${WLS:-c3 c5}; do
for v in 0 1; do
  if [ $v = 1 ]; then cmd="env $SW"; else cmd=""; fi
  $cmd timeout -k 10 400 python -u bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/${w}_$v.json 2> $OUT/${w}_$v.err || { echo "$w failed"; tail -5 $OUT/${w}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/${w}_$v.json')); r=d['roofline']; c=d['config']; t=d['trial_kernel_ms']
print('$w', 'sw=$v', round(d['value'],3), r['tiles'], r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'], r['frac_survey'], t.get('sp_glin_rows'), c['chi2_final'])"
done
done
