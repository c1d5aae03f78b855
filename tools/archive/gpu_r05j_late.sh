#!/bin/bash
# the device-driven LM on the final build: same-box A/B against the host loop
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05j
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - DEFTRI_DEVICE_LM=1 - DEFTRI_DEVICE_LM=1 > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('pts_sum'), d.get('trials'))
"
