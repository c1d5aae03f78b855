#!/bin/bash
# round 3: iterative-plan parity tests, then N alternating C2 bench runs of the default build (value, CG iteration, frac, phases)
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_sp.py tests/test_c2_golden.py tests/test_regime_goldens.py} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in ${RUNS:-a b}; do
  case $v in x*) E="${XENV:-}";; *) E="";; esac
  env $E timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b_$v.json 2> $OUT/b_$v.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', '$E', round(d['value'],1), r['cg_iteration_us'], r['frac'], r['phase1']['us'], r['phase2']['us'])"
done
