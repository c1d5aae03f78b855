#!/bin/bash
# the trial's wait by stream polling: same-box A/B, and the trace's gaps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05h
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - DEFTRI_SYNC_BLOCK=1 - DEFTRI_SYNC_BLOCK=1 > $OUT/ab.log 2>&1 || { echo ab failed; tail -30 $OUT/ab.log; exit 1; }
python3 -c "
import json
for l in open('$OUT/ab.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('env'), d.get('lm_it_s'), d.get('cg_iteration_us'), d.get('repeat_same'), d.get('pts_sum'))
"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e --no-legs --trace-markers > $OUT/prof.json 2> $OUT/prof.err || { echo trace failed; tail -5 $OUT/prof.err; exit 1; }
cd $R && python3 tools/trace_gaps.py $OUT/prof/run_kernel_trace.csv --window MulFunctor | tail -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_sp.py tests/test_c2_golden.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
