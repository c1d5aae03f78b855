#!/bin/bash
# PCG GPU tests + one C2 bench line (no CPU baseline, no end-to-end) with a summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pcg}
mkdir -p $OUT
cd $R
if [ -n "${TESTS:-tests/test_gpu_pcg.py}" ]; then
  timeout -k 10 ${TLIM:-500} python3 -u -m pytest ${TESTS:-tests/test_gpu_pcg.py} -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  grep -E "PASS|FAIL|ERROR|^E  " $OUT/pytest.log | grep -v "array(" | tail -30
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); c=d['config']
print('value', round(d['value'],2), 'ms/trial', c['ms_per_trial'], 'cg/trial', c.get('cg_iterations_per_pcg_trial'), 'fallbacks', c.get('pcg_fallbacks'))
print('roofline', d['roofline'])
print('trial_kernel_ms', d['trial_kernel_ms'])
print('breakdown', d['breakdown_ms'])"
