#!/bin/bash
# round 3 final build: the whole -m gpu suite, smoke, the headline measurement pass (bench + rocprofv3 stats + PMC), a trace
set -o pipefail
OUT=gpurun_out/${1:-r03z}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/r03_prof.sh ${1:-r03z}
