#!/bin/bash
# round 6, closing measurement: the drop-in call's host stages at C2, the default bench line (C2 headline,
# CPU baseline, end-to-end, 500k and Realcolon legs) and its rocprofv3 kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06f3}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
DEFTRI_CALL_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_GRAPH_TIMING=1 DEFTRI_UPLOAD_TIMING=1 \
  timeout -k 10 300 python -u tools/e2e_timing.py 100000 > $OUT/e2e.log 2>&1 || { echo "e2e failed"; tail -20 $OUT/e2e.log; exit 1; }
grep -E "deftri call|slot scan|plan [0-9]" $OUT/e2e.log | tail -8
timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));r=d['roofline'];e=d['config'].get('end_to_end_arap_optimization',{});print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac_survey'], r['cg_iteration_us'], d['cpu_baseline']['value'], e.get('next_round_call_s'), e.get('warm_call_s'), e.get('cold_call_s'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-legs > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
echo prof ok
