#!/bin/bash
# round-5 lines of the multi-keyframe workloads (BASELINE C3-C5) on the final build, and the host
# round-trip timing at C2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05k
mkdir -p $OUT
cd $R
DEFTRI_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e --no-legs > $OUT/c2_host_timing.json 2> $OUT/c2_host_timing.err || { echo c2 failed; tail -5 $OUT/c2_host_timing.err; exit 1; }
grep "deftri host" $OUT/c2_host_timing.err | tail -3
for w in c3 c5 c4; do
  timeout -k 10 900 python -u bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo $w failed; tail -20 $OUT/bench_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$w.json'));print('$w', round(d['value'],3), round(d['ms_per_step'],2), d['config'].get('cg_iterations_per_pcg_trial'))"
done
