#!/bin/bash
# A/B of library builds on the C2 bench (same box, alternating): LIBS="a.so b.so" (paths relative to the package)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ablib}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for L in ${LIBS}; do
    n=$(basename $L .so)
    DEFTRI_LIB=$R/triangulation-in-deformable-scenes_amd/$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e > $OUT/bench_${n}_$rep.json 2> $OUT/bench_${n}_$rep.err
    python3 -c "import json; d=json.load(open('$OUT/bench_${n}_$rep.json')); print('$n', $rep, round(d['value'],1), 'it/s', d['roofline']['avg_active_launch_us'], 'us')"
  done
done
