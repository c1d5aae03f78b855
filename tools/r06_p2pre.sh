#!/bin/bash
# round 6: k_sp_tile's per-row pass with its depth coupling (several pairs: G.tdep) and diagonal block
# loaded in the prologue (working tree) against ab/libdeftri_base.so: C2 / 500k on tools/tile_ab.py,
# C3 and C5 on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06p2pre}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
for n in 100000 500000; do
  timeout -k 10 400 python -u tools/tile_ab.py $n 10 DEFTRI_LIB=$B - DEFTRI_LIB=$B - > $OUT/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -5 $OUT/ab_$n.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$OUT/ab_$n.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print($n, d['env'], d['cg_us'], d['cg_iteration_us'], d['lm_it_s'])
    elif l.startswith('{\"same'): print(l.strip())
"
done
for w in c3 c5; do
for v in $B ""; do
  DEFTRI_LIB=${v:-$R/triangulation-in-deformable-scenes_amd/libdeftri.so} timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail -5 $OUT/$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$w.json')); r=d['roofline']; c=d['config']
print('$w', '${v:-tree}'.split('/')[-1], r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'], c['chi2_final'])"
done
done
