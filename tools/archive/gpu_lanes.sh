#!/bin/bash
# Speculative-lane check: bit-identity tests, then the C2 bench at several lane counts.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-lanes}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "lanes" > $OUT/pytest_lanes.log 2>&1 || { tail -60 $OUT/pytest_lanes.log; exit 1; }
tail -6 $OUT/pytest_lanes.log
for n in ${LANES:-1 2 3 4}; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --lanes $n > $OUT/bench_l$n.json 2> $OUT/bench_l$n.err || { tail -30 $OUT/bench_l$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value'],2), d['ms_per_step'], d['config']['lm_lanes'], d['config']['trials_per_iteration'], d['config']['trials_executed_per_iteration'])" $OUT/bench_l$n.json
done
