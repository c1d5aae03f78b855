#!/bin/bash
# round 6: host stages of the drop-in call at C2 (cold / warm / next round) and of C4's upload, with the
# library's stage timers; then the tile-plan GPU tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06up2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export DEFTRI_CALL_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_GRAPH_TIMING=1 DEFTRI_UPLOAD_TIMING=1
timeout -k 10 300 python -u tools/e2e_timing.py 100000 > $OUT/e2e.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e.log; exit 1; }
grep -E "deftri (call|upload)|4a tiles  |next_round" $OUT/e2e.log | tail -12
timeout -k 10 400 python -u bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail -20 $OUT/c4.err; exit 1; }
grep -E "4a [a-z]|plan [0-9]|upload" $OUT/c4.err | grep -v "4a tiles [0-9]" | head -20
unset DEFTRI_CALL_TIMING DEFTRI_PLAN_TIMING DEFTRI_GRAPH_TIMING DEFTRI_UPLOAD_TIMING
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sp.py tests/test_c2_golden.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
