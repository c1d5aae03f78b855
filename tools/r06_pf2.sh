#!/bin/bash
# round 6: the next entry pass's J prefetched during the current one (163 VGPRs, 3 waves per SIMD) against
# the committed build: C2 and 500k x 2 on tools/tile_ab.py, C3 on bench.py
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06pf2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
V=$R/ab/libdeftri_pf2.so
for n in 100000 500000; do
  timeout -k 10 400 python -u tools/tile_ab.py $n 10 DEFTRI_LIB=$B DEFTRI_LIB=$V DEFTRI_LIB=$B DEFTRI_LIB=$V > $OUT/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -5 $OUT/ab_$n.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$OUT/ab_$n.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print($n, d['env'], d['tiles'], d['cg_us'], d['cg_iteration_us'], d['lm_it_s'], d['pcg_its'])
    elif l.startswith('{\"same'): print(l.strip())
"
done
for v in $B $V; do
  DEFTRI_LIB=$v timeout -k 10 300 python -u bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail -5 $OUT/c3.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/c3.json')); r=d['roofline']
print('c3', '$v'.split('/')[-1], r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'])"
done
