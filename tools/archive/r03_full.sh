#!/bin/bash
# round 3: the whole -m gpu suite, then the C2 A/B (fused / unfused) and a kernel trace
set -o pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
SKIP_AB_TESTS=1 bash tools/r03_ab.sh
