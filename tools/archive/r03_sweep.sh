#!/bin/bash
# round 3: iterative-plan tests, then C2 / C3 / C5 / C4 bench lines without CPU baselines
set -o pipefail
OUT=gpurun_out/${1:-r03s}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sp.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
for w in c2 c3 c5 c4; do
  timeout -k 10 500 python -u bench.py --workload $w --steps $([ $w = c2 ] && echo 25 || echo 5) --no-cpu-baseline --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo $w failed; tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));r=d['roofline'];print('$w', round(d['value'],2), r['cg_iteration_us'], r['frac'], r['phase1']['us'], r['phase2']['us'])"
done
