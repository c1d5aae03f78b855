#!/bin/bash
# round 3: A/B of an env switch on the C2 bench (alternating), then a kernel trace of the default
set -o pipefail
OUT=gpurun_out/r03ab2
mkdir -p $OUT
VAR="$1"
for v in a b a2 b2; do
  case $v in a*) E="";; b*) E="$VAR";; esac
  env $E timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/ab_$v.json 2> $OUT/ab_$v.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/ab_$v.json').read().strip().splitlines()[-1]);print('$v', '$E', round(d['value'],1), d['config']['ms_per_cg_iteration_profiled'])"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e --trace-markers > $R/$OUT/prof.json 2> $R/$OUT/prof.err || { echo trace failed; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt
