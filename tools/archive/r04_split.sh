#!/bin/bash
# round 4: lane-pair wave split (spcg_plan.cpp 8b) — GPU tests of the iterative plan, phase-2 wave
# trace, same-box A/B of the split threshold and the rows' linearization step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04sp}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sp.py tests/test_c2_golden.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
i=0
for e in "" "DEFTRI_SP_WAVE_SPLIT=0"; do
  i=$((i+1))
  env $e DEFTRI_SP_P2_TRACE=$OUT/tr_$i.bin timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "run $i failed"; tail -5 $OUT/b_$i.err; exit 1; }
  echo "== [$e]"; python tools/p2trace.py $OUT/tr_$i.bin $OUT/tr_$i.json > /dev/null && python -c "
import json;d=json.load(open('$OUT/tr_$i.json'));print({k:d[k] for k in ('waves','span_us','slot_loop_us','wave_life_us','end_us','steps')})"
done
TAG=${TAG:-r04sp}ab bash tools/r04_ab.sh "" "DEFTRI_SP_GLIN_STEP=6" "DEFTRI_SP_WAVE_SPLIT=0" "DEFTRI_ARAP_J_FULL=1"
