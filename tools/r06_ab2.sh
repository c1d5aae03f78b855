#!/bin/bash
# round 6: the working tree's build against ab/libdeftri_base.so at C2 (tools/tile_ab.py: the LM run,
# the profiled trial's linearization, CG and per-trial kernels)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06ab2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
timeout -k 10 400 python -u tools/tile_ab.py ${N:-100000} 10 DEFTRI_LIB=$B - DEFTRI_LIB=$B - > $OUT/ab.log 2>&1 || { echo "ab failed"; tail -5 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print(d['env'], d['lm_it_s'], d['cg_iteration_us'], d['lin_us'], d['trial_us'])
    elif l.startswith('{\"same'): print(l.strip())
"
