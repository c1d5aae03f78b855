#!/bin/bash
# round 4: selected -m gpu tests (arg 2: pytest -k / file list), then the C2 bench line without the CPU leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04a}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread ${2:-tests} > $OUT/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/pytest.log | tail -60
tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac'], r['cg_iteration_us'], d['config']['trials_per_iteration'], d['config']['cg_iterations_per_pcg_trial'], d['end_to_end_arap_optimization'])"
exit $rc
