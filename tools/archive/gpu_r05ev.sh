#!/bin/bash
# the fused trial evaluation: same-box A/B against the split launches, edges per thread, then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ev
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - DEFTRI_EVAL_SPLIT=1 DEFTRI_EVAL_EPT=2 DEFTRI_EVAL_EPT=8 - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('trial_us'), d.get('trials'), d.get('repeat_same'))
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
