#!/bin/bash
# SQ wave-state counters for the PCG kernels over a short C2 bench run (one rocprofv3 pass).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sqpcg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/sq.json 2> $OUT/sq.err
ls $OUT/sq
