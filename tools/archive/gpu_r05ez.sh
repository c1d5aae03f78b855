#!/bin/bash
# the row pass's slot stream: same-box A/B (row-pass step variants), then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ez
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u tools/tile_ab.py 100000 25 - DEFTRI_SP_SLOT_STREAM=0 DEFTRI_SP_GLIN_STEP=6 DEFTRI_SP_GLIN_STEP=8 DEFTRI_EVAL_SPLIT=1,DEFTRI_SP_SLOT_STREAM=0 - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('lin_us'), d.get('trial_us'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('pts_sum'))
"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
