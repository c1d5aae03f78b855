#!/bin/bash
# round 6: A/B of the working tree's build against ab/libdeftri_base.so (C2, 500k x 2), then the GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06abchk}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
bash tools/r06_ab.sh $TAG || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
