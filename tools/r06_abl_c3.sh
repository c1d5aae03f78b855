set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06abl_c3
mkdir -p $OUT
cd $R
for v in base NOALPHA; do
  DEFTRI_LIB=$R/ab/libdeftri_$v.so timeout -k 10 300 python -u bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$v.json 2> $OUT/$v.err || { echo "$v failed"; tail -5 $OUT/$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$v.json')); r=d['roofline']; print('$v', r['phase1'], r['phase2'], r['cg_iteration_us'])"
done
