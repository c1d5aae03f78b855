#!/bin/bash
# GPU tests + C2 bench A/B of environment toggles (no CPU baseline).  AB="NAME=VAL ..." settings,
# each run once against the default.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TLIM:-600} python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); t=d.get('factorization_trial_kernel_ms') or d['trial_kernel_ms']; c=d['config']; r=d['roofline']; print(sys.argv[2], round(d['value'],2), 'ms/trial', c['ms_per_trial'], 'solver', c.get('step_solver'), 'cg/trial', c.get('cg_iterations_per_pcg_trial'), 'fallbacks', c.get('pcg_fallbacks'), r['kernel'], r['achieved'], r['unit'], 'frac', r['frac'], 'upd', t['update'], 'trsm', t.get('trsm'), 'diag', t['diag'])" "$@"; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/base.json 2> $OUT/base.err || { tail -30 $OUT/base.err; exit 1; }
summ $OUT/base.json base
for kv in ${AB:-}; do
  tag=$(echo "$kv" | tr '/=' '__')
  env $kv timeout -k 10 300 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/ab_$tag.json 2> $OUT/ab_$tag.err || { tail -30 $OUT/ab_$tag.err; exit 1; }
  summ $OUT/ab_$tag.json $kv
done
