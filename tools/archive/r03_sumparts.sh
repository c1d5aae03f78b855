#!/bin/bash
# round 3: fused chi2-sum workgroups per job (DEFTRI_SP_SUM_PARTS) A/B on C2 under rocprofv3 --stats
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03sp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 128 256 512 64; do
  DEFTRI_SP_SUM_PARTS=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b$v.json 2> $OUT/b$v.err || { echo run $v failed; tail -5 $OUT/b$v.err; exit 1; }
  python3 -c "
import csv,json
d=json.loads(open('$OUT/b$v.json').read().strip().splitlines()[-1])
st={r['Name'][:40]:float(r['AverageNs'])/1e3 for r in csv.DictReader(open('$OUT/p$v/run_kernel_stats.csv'))}
print('$v', round(d['value'],1), {k:round(x,2) for k,x in st.items() if 'sum_multi' in k or 'lin_chi' in k})"
done
