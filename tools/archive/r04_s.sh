#!/bin/bash
# round 4: CG state recorded by phase 2 (no tail launch), setup at 6 waves/SIMD — GPU tests of the
# iterative plan, A/B line, and the timed loop's kernel-trace gaps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04s}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sp.py tests/test_c2_golden.py tests/test_full_size_props.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=${TAG:-r04s} bash tools/r04_ab.sh ""
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 1 --no-cpu-baseline --no-e2e --trace-markers > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
cd $R && python tools/trace_gaps.py $OUT/prof --window MulFunctor --json $OUT/gaps.json > $OUT/gaps.txt && head -30 $OUT/gaps.txt
