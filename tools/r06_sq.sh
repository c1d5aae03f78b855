#!/bin/bash
# round 6: SQ counters (occupancy, issue, waits, LDS) of the tile-mode CG kernels k_sp_tile / k_sp_tupd
# at C2 and at 500k x 2.  One rocprofv3 pass per counter group (kernel trace only, no other domains),
# each under its own time limit; the summary is made on the CPU afterwards (tools/pmc_sq_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06sq}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
for corr in 100000 500000; do
  i=0
  for G in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G --kernel-trace --output-format csv -d $OUT/c${corr}_g$i -o run -- \
      python3 $R/bench.py --corr $corr --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-legs \
      > $OUT/c${corr}_g$i.json 2> $OUT/c${corr}_g$i.err || { echo "pass c$corr g$i failed"; tail -5 $OUT/c${corr}_g$i.err; exit 1; }
    echo "pass c$corr g$i ok"
  done
done
