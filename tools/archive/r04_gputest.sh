#!/bin/bash
# round 4: the whole GPU suite and the smoke, logs under gpurun_out/<tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04t}
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
