#!/bin/bash
# the round's final build: the GPU suite, then the measurement pass (bench, rocprof, PMC)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r05i
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05i/pytest.log 2>&1 || { echo pytest failed; grep -E "FAILED|Error" gpurun_out/r05i/pytest.log | head -20; tail -5 gpurun_out/r05i/pytest.log; exit 1; }
tail -2 gpurun_out/r05i/pytest.log
bash tools/r05_measure.sh r05i
