#!/bin/bash
# phase-2 wave timelines at C2 (DEFTRI_SP_P2_TRACE): default, 4-slot steps, row split 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04tr}
mkdir -p $OUT
cd $R
i=0
for e in "" "DEFTRI_SP_P2_STEP=4" "DEFTRI_SP_ROW_SPLIT=2 DEFTRI_SP_P2_STEP=4" "DEFTRI_SP_ALPHA_KERNEL=1"; do
  i=$((i+1))
  env $e DEFTRI_SP_P2_TRACE=$OUT/tr_$i.bin timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/b_$i.json 2> $OUT/b_$i.err || { echo "run $i failed"; tail -5 $OUT/b_$i.err; exit 1; }
  echo "== [$e]"; python tools/p2trace.py $OUT/tr_$i.bin $OUT/tr_$i.json
done
