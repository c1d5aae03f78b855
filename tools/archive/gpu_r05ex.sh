#!/bin/bash
# host-finished evaluation sums and the folded trial prologue: same-box A/B, regime-golden deviations,
# then the GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ex
mkdir -p $OUT
cd $R
OLD=DEFTRI_EVAL_SPLIT=1,DEFTRI_SP_SETUP_DOF=1
timeout -k 10 500 python -u tools/tile_ab.py 100000 25 - DEFTRI_TRIAL_BEGIN=1 DEFTRI_EVAL_EPT=1 DEFTRI_EVAL_EPT=2 DEFTRI_EVAL_EPT=8 DEFTRI_EVAL_DEVICE_SUMS=1 $OLD - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('trial_us'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('trials')==None)
"
timeout -k 10 300 python -u tools/regime_dev.py realcolon regimes - DEFTRI_TRIAL_BEGIN=1 DEFTRI_EVAL_EPT=1 DEFTRI_EVAL_EPT=2 DEFTRI_EVAL_EPT=8 DEFTRI_EVAL_DEVICE_SUMS=1 > $OUT/dev_rc.log 2>&1 || { echo dev failed; tail -30 $OUT/dev_rc.log; exit 1; }
cat $OUT/dev_rc.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
