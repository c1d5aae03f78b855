#!/bin/bash
# round 4: the trial's evaluation fused into two launches — GPU tests of the iterative plan, A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04ev}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sp.py tests/test_c2_golden.py tests/test_regime_goldens.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=${TAG:-r04ev} bash tools/r04_ab.sh "" "DEFTRI_NO_EVAL_FUSE=1"
