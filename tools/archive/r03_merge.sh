#!/bin/bash
# round 3: merged CG chain (2 launches) — iterative-plan parity tests, then A/B vs the 3-launch chain on C2 and a trace
set -o pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_sp.py tests/test_regime_goldens.py tests/test_c2_golden.py} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in a b a2 b2; do
  case $v in a*) E="";; b*) E="DEFTRI_SP_NO_MERGE=1";; esac
  env $E timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/ab_$v.json 2> $OUT/ab_$v.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/ab_$v.json').read().strip().splitlines()[-1]);print('$v', '$E', round(d['value'],1), d['config']['ms_per_cg_iteration_profiled'], d['roofline']['frac'])"
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e --trace-markers > $R/$OUT/prof.json 2> $R/$OUT/prof.err || { echo trace failed; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt && cat $OUT/gaps.txt | head -8
