#!/bin/bash
# phase-2 wave timelines at C2 (DEFTRI_SP_P2_TRACE): default, 4-slot steps, row split 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04tr}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sp.py -k step_size > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
i=0
for e in "" "DEFTRI_SP_P2_STEP=6"; do
  i=$((i+1))
  env $e DEFTRI_SP_P2_TRACE=$OUT/tr_$i.bin timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "run $i failed"; tail -5 $OUT/b_$i.err; exit 1; }
  echo "== [$e]"; python tools/p2trace.py $OUT/tr_$i.bin $OUT/tr_$i.json
done
TAG=${TAG:-r04tr}ab bash tools/r04_ab.sh "" "DEFTRI_SP_P2_STEP=6 DEFTRI_SP_GLIN_STEP=6" "DEFTRI_SP_P2_STEP=6" "DEFTRI_SP_GLIN_STEP=6"
