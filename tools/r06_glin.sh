#!/bin/bash
# round 6: k_sp_glin_rows' depth edges four at a time (working tree) against ab/libdeftri_base.so: the
# profiled trial's linearization kernels at C2 (tools/tile_ab.py) and C3 / C5 (bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06glin}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B=$R/ab/libdeftri_base.so
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 DEFTRI_LIB=$B - DEFTRI_LIB=$B - > $OUT/ab_c2.log 2>&1 || { echo "ab failed"; tail -5 $OUT/ab_c2.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab_c2.log'):
    if l.startswith('{\"tiles'):
        d=json.loads(l); print('c2', d['env'], d['lin_us'], d['lm_it_s'])
    elif l.startswith('{\"same'): print(l.strip())
"
for w in c3 c5; do
for v in $B ""; do
  DEFTRI_LIB=${v:-$R/triangulation-in-deformable-scenes_amd/libdeftri.so} timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; tail -5 $OUT/$w.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$w.json')); t=d['trial_kernel_ms']; c=d['config']
print('$w', '${v:-tree}'.split('/')[-1], t.get('sp_glin_rows'), t.get('lin_arap'), round(d['value'],3), c['chi2_final'])"
done
done
