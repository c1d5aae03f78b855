#!/bin/bash
# the linearization's chi2 from its workgroups' partials: same-box A/B, Realcolon golden deviation, GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05f
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - DEFTRI_LIN_CHI_ARRAYS=1 - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('lin_us'), d.get('trial_us'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('pts_sum'))
"
timeout -k 10 300 python -u tools/regime_dev.py realcolon regimes - DEFTRI_LIN_CHI_ARRAYS=1 > $OUT/dev_rc.log 2>&1 || { echo dev failed; tail -30 $OUT/dev_rc.log; exit 1; }
cat $OUT/dev_rc.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
