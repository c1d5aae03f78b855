#!/bin/bash
# SQ counters per k_update dispatch (one rocprofv3 --pmc pass, kernel trace only), C2, 2 LM iterations.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-squ}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 --kernel-include-regex "k_update|k_trsm|k_diag" --kernel-trace --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/lane_trace.py 100000 1 2 > $OUT/sq.txt 2>&1
ls $OUT/pmc
