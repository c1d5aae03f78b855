#!/bin/bash
# edges per thread 2; the setup variants against the sharded oracle test and the Realcolon golden; A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05ey
mkdir -p $OUT
cd $R
K="test_sharded_iterative_matches_oracle or (test_regime_matches_oracle and realcolon-regimes-iterative)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_sp.py tests/test_regime_goldens.py -m gpu -v --timeout 200 --timeout-method thread -k "$K" > $OUT/t_row.log 2>&1; echo "row setup rc=$?"; grep -E "PASSED|FAILED|rel" $OUT/t_row.log | head -20
DEFTRI_SP_SETUP_DOF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_sp.py tests/test_regime_goldens.py -m gpu -v --timeout 200 --timeout-method thread -k "$K" > $OUT/t_dof.log 2>&1; echo "dof setup rc=$?"; grep -E "PASSED|FAILED|rel" $OUT/t_dof.log | head -20
OLD=DEFTRI_EVAL_SPLIT=1,DEFTRI_SP_SETUP_DOF=1
timeout -k 10 500 python -u tools/tile_ab.py 100000 25 - DEFTRI_TRIAL_BEGIN=1 DEFTRI_SP_SETUP_DOF=1 $OLD - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('trial_us'), d.get('cg_iteration_us'), d.get('repeat_same'))
"
