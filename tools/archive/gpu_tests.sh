#!/bin/bash
# GPU tests (given files or the whole -m gpu suite), one process, per-test timeout.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-tests}
mkdir -p $OUT
cd $R
timeout -k 10 ${TLIM:-900} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -80 $OUT/pytest_gpu.log; exit 1; }
tail -25 $OUT/pytest_gpu.log
