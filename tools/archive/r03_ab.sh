#!/bin/bash
# round 3: CG-chain A/B (fused / unfused) on C2 + kernel trace of the fused timed loop
set -o pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
export PYTHONUNBUFFERED=1
[ -n "$SKIP_AB_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sp.py tests/test_regime_goldens.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
for v in "fused" "unfused DEFTRI_SP_NO_FUSE=1" "fused2" "unfused2 DEFTRI_SP_NO_FUSE=1"; do
  set -- $v
  env $2 timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/ab_$1.json 2> $OUT/ab_$1.err || exit 1
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e --trace-markers > $R/$OUT/prof.json 2> $R/$OUT/prof.err || { echo trace failed; tail -5 $R/$OUT/prof.err; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt
