#!/bin/bash
# round 3: iterative-plan parity tests, then the C2 bench under rocprofv3 --stats twice (value + per-kernel means)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r03ck
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sp.py tests/test_c2_golden.py tests/test_regime_goldens.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in a b; do
  timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/v$v.json 2> $OUT/v$v.err || exit 1
  python -c "import json;d=json.loads(open('$OUT/v$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', round(d['value'],1), r['cg_iteration_us'], r['frac'], r['phase1']['us'], r['phase2']['us'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/b.json 2> $OUT/b.err || { echo prof failed; tail -5 $OUT/b.err; exit 1; }
python3 -c "
import csv
st={r['Name'].split('(')[0].split('::')[-1][:22]:float(r['AverageNs'])/1e3 for r in csv.DictReader(open('$OUT/p/run_kernel_stats.csv'))}
print({k:round(x,1) for k,x in st.items() if any(t in k for t in ('phase','glin_rows','lin_chi','lin_arap','sum_multi','setup'))})"
