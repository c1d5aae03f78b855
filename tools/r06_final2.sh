#!/bin/bash
# round 6, last pass: the drop-in call's host stages at C2 (stage timers), then the whole GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06f2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
DEFTRI_CALL_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_GRAPH_TIMING=1 DEFTRI_UPLOAD_TIMING=1 \
  timeout -k 10 300 python -u tools/e2e_timing.py 100000 > $OUT/e2e.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e.log; exit 1; }
grep -E "deftri call|free device|plan [0-9]|4a tiles  |keyframe|delaunay" $OUT/e2e.log | tail -14
tail -1 $OUT/e2e.log
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
