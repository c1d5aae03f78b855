#!/bin/bash
# round 6: the whole GPU test suite (no -x: every failure listed), then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06full}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit 1; fi
if [ -n "${NO_BENCH:-}" ]; then exit 0; fi
timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));r=d['roofline'];print('C2', round(d['value'],1), round(d['ms_per_step'],4), r['frac_survey'], r['cg_iteration_us'], d['cpu_baseline']['value'])"
