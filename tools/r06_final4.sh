#!/bin/bash
# round 6, closing pass on the final tree: the whole GPU suite, then the measurement of r06_final3.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06f4}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 800 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/r06_final3.sh $TAG
