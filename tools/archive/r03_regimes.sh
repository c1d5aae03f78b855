#!/bin/bash
# round 3: the C2 scene under the Drunkard and Realcolon weights, PCG (iterative plan) vs LDL^T
# (multifrontal plan, direct steps), plus the C5-shape parity tests
set -o pipefail
OUT=gpurun_out/${1:-r03r}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sp.py -k c5_shape > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
for rg in drunkard realcolon; do
  timeout -k 10 400 python -u bench.py --regime $rg --no-cpu-baseline > $OUT/bench_$rg.json 2> $OUT/bench_$rg.err || { echo $rg failed; tail -20 $OUT/bench_$rg.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$rg.json'));c=d['config'];print('$rg pcg', round(d['value'],1), c['trials_per_iteration'], c['ms_per_trial'], c['pcg_trials'], c['pcg_failed_or_fallback'], c['cg_iterations_per_pcg_trial'])"
  timeout -k 10 400 python -u bench.py --regime $rg --plan multifrontal --solver direct --no-cpu-baseline > $OUT/bench_${rg}_ldlt.json 2> $OUT/bench_${rg}_ldlt.err || { echo $rg ldlt failed; tail -20 $OUT/bench_${rg}_ldlt.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_${rg}_ldlt.json'));c=d['config'];print('$rg ldlt', round(d['value'],1), c['trials_per_iteration'], c['ms_per_trial'])"
done
