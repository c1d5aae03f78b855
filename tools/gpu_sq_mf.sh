#!/bin/bash
# SQ instruction-mix / LDS counters for the matrix-free PCG kernels over a short C2 bench run (one
# rocprofv3 pass, counters only with --kernel-trace).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sqmf}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/sq.json 2> $OUT/sq.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/sq2.json 2> $OUT/sq2.err
ls $OUT/sq $OUT/sq2
