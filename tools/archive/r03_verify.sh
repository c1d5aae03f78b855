#!/bin/bash
# round 3 re-entry: the whole -m gpu suite, smoke, then the flat / grouped ticket A/B on C2 and a kernel trace
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
bash tools/r03_ab2.sh DEFTRI_FLAT_TICKET=1
