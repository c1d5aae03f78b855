#!/bin/bash
# round 6: the update's share-plane and cross-slot loads four at a time (working tree) against the
# committed build (ab/libdeftri_base.so): C2 / 500k on tools/tile_ab.py, C3 and C5 on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06tupd}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 DEFTRI_LIB=$B - DEFTRI_LIB=$B - > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -5 $OUT/ab_c2.log; exit 1; }
grep -h '"same' $OUT/ab_c2.log
for w in c3 c5; do
for v in $B ""; do
  DEFTRI_LIB=${v:-$R/triangulation-in-deformable-scenes_amd/libdeftri.so} timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail -5 $OUT/$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$w.json')); r=d['roofline']; c=d['config']
print('$w', '${v:-tree}'.split('/')[-1], r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'], c['chi2_final'])"
done
done
