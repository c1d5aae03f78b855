#!/bin/bash
# the update's heavy partials in one batch: same-box A/B against the previous build, the solver tests
# previous build (ab/libdeftri_base.so), the solver tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05q
mkdir -p $OUT
cd $R
B=DEFTRI_LIB=$R/ab/libdeftri_base.so
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - $B - $B > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('cg_us'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('pts_sum'))
"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sp.py tests/test_c2_golden.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
