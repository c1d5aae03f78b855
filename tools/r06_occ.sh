#!/bin/bash
# round 6: k_sp_tile at 4 / 5 / 6 waves per SIMD (ab/libdeftri_w*.so) with LDS budgets that let 5 / 6
# workgroups share a CU; C2 and 500k x 2 on tools/tile_ab.py, C3 on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06occ}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
for n in 100000 500000; do
  timeout -k 10 400 python -u tools/tile_ab.py $n 10 DEFTRI_LIB=$B - DEFTRI_LIB=$B,DEFTRI_SP_TILE_LDS=31744 DEFTRI_LIB=$R/ab/libdeftri_w5.so,DEFTRI_SP_TILE_LDS=31744 DEFTRI_LIB=$R/ab/libdeftri_w6.so,DEFTRI_SP_TILE_LDS=26112 > $OUT/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -5 $OUT/ab_$n.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$OUT/ab_$n.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print($n, d['env'], d['tiles'], d['cg_us'], d['cg_iteration_us'], d['lm_it_s'], d['pcg_its'])
    elif l.startswith('{\"same'): print(l.strip())
"
done
for v in "DEFTRI_LIB=$B" "DEFTRI_LIB=$R/ab/libdeftri_w5.so DEFTRI_SP_TILE_LDS=31744"; do
  env $v timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 1 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail -5 $OUT/c3.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c3.json')); r=d['roofline']; c=d['config']
print('c3', '$v'.split('/')[-1], round(d['value'],3), r.get('frac_survey'), r.get('cg_iteration_us'), r.get('tiles'), r['phase1']['us'], r['phase2']['us'], c.get('cg_iterations_per_pcg_trial'))"
done
