#!/bin/bash
# round 3: row-sort A/B (DEFTRI_SP_NO_ROWSORT=1) on C2 under rocprofv3 --stats: per-kernel means and the value
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03rs
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in s n s2 n2; do
  case $v in n*) E="DEFTRI_SP_NO_ROWSORT=1";; *) E="DEFTRI_SP_X=0";; esac
  env $E timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p$v -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b$v.json 2> $OUT/b$v.err || { echo run $v failed; tail -5 $OUT/b$v.err; exit 1; }
  python3 -c "
import csv,json
d=json.loads(open('$OUT/b$v.json').read().strip().splitlines()[-1])
st={r['Name'].split('(')[0].split('::')[-1][:22]:float(r['AverageNs'])/1e3 for r in csv.DictReader(open('$OUT/p$v/run_kernel_stats.csv'))}
print('$v', round(d['value'],1), {k:round(x,1) for k,x in st.items() if any(t in k for t in ('phase','glin_rows','lin_chi','lin_arap','sum_multi','setup'))})"
done
