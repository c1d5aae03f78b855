#!/bin/bash
# SQ stall / MFMA-busy counters for the bench's kernels (one rocprofv3 pass, kernel trace only).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.json 2> $OUT/sq.err
ls $OUT/sq
