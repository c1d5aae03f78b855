#!/bin/bash
# A/B of the matrix-free slice height (DEFTRI_MF_ROWS) on the C2 bench, one process per setting.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-mfrows}
mkdir -p $OUT
cd $R
for r in ${ROWS:-64 48 40 32}; do
  DEFTRI_MF_ROWS=$r timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e > $OUT/bench_$r.json 2> $OUT/bench_$r.err
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$r.json')); print('rows $r', round(d['value'],1), 'it/s', d['roofline']['avg_active_launch_us'], 'us', d['roofline']['bytes_per_launch'])"
done
