#!/bin/bash
# round 3: the whole -m gpu suite, smoke, then the merged / three-launch C2 A/B and a kernel trace (r03_merge.sh)
set -o pipefail
OUT=gpurun_out/r03f2
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
TESTS="tests/test_gpu_sp.py -k merged" bash tools/r03_merge.sh
