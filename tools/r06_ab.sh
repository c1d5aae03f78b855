#!/bin/bash
# round 6 A/B: the committed build (ab/libdeftri_base.so) against the working tree's, same box,
# tools/tile_ab.py (C2 and 500k x 2: LM run, profiled trial's CG kernels on HIP events)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06ab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for n in 100000 500000; do
  timeout -k 10 300 python -u tools/tile_ab.py $n 10 DEFTRI_LIB=$R/ab/libdeftri_base.so - DEFTRI_LIB=$R/ab/libdeftri_base.so - > $OUT/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -5 $OUT/ab_$n.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$OUT/ab_$n.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print($n, d['env'], d['cg_us'], d['cg_iteration_us'], d['lm_it_s'], d['trials'][:4], d['pcg_its'])
    elif l.startswith('{\"same'): print(l.strip())
"
done
