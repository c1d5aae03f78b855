#!/bin/bash
# the heavy partials' loads four edges at a time: timing and bit-identity, the solver tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05l
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u tools/tile_ab.py 100000 25 - - > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('lin_us'), d.get('repeat_same'), d.get('pts_sum'))
"
timeout -k 10 600 python -u -m pytest tests/test_gpu_sp.py tests/test_c2_golden.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
