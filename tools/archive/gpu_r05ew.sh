#!/bin/bash
# the one-thread-per-row setup and the fused evaluation: regime-golden deviations per variant, same-box A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ew
mkdir -p $OUT
cd $R
OLD=DEFTRI_EVAL_SPLIT=1,DEFTRI_SP_SETUP_DOF=1
timeout -k 10 300 python -u tools/regime_dev.py realcolon regimes $OLD - DEFTRI_EVAL_SPLIT=1 DEFTRI_SP_SETUP_DOF=1 DEFTRI_EVAL_EPT=8 > $OUT/dev_rc.log 2>&1 || { echo dev failed; tail -30 $OUT/dev_rc.log; exit 1; }
cat $OUT/dev_rc.log
for g in simulation drunkard; do
  timeout -k 10 200 python -u tools/regime_dev.py $g regimes $OLD - DEFTRI_EVAL_EPT=8 > $OUT/dev_$g.log 2>&1 || { echo dev $g failed; tail -30 $OUT/dev_$g.log; exit 1; }
  cat $OUT/dev_$g.log
done
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - $OLD DEFTRI_SP_SETUP_DOF=1 DEFTRI_EVAL_EPT=8 - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('trial_us'), d.get('cg_iteration_us'), d.get('repeat_same'))
"
