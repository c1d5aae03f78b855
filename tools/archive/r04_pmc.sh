#!/bin/bash
# round 4 counter passes (each its own rocprofv3 run, counters within one block's limits):
#   1. FETCH_SIZE / WRITE_SIZE calibration of the access widths the CG kernels use (tools/micro/fetch_calib)
#   2. SQ wave-state counters of the CG kernels at C2 (phase 2's wait / issue split)
#   3. TCC hit / miss of the CG kernels at C2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/cal_fetch -o run -- $R/tools/micro/fetch_calib > $OUT/cal_fetch.log 2>&1 || { echo cal fetch failed; tail -5 $OUT/cal_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/cal_write -o run -- $R/tools/micro/fetch_calib > $OUT/cal_write.log 2>&1 || { echo cal write failed; tail -5 $OUT/cal_write.log; exit 1; }
python3 $R/tools/micro/fetch_calib_summary.py $OUT/cal_fetch/run_counter_collection.csv $OUT/cal_write/run_counter_collection.csv $OUT/fetch_calibration.json | head -12
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/sq.json 2> $OUT/sq.err || { echo sq failed; tail -5 $OUT/sq.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/tcc -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/tcc.json 2> $OUT/tcc.err || { echo tcc failed; tail -5 $OUT/tcc.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || { echo fetch failed; tail -5 $OUT/pmc_fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmc_write.json 2> $OUT/pmc_write.err || { echo write failed; tail -5 $OUT/pmc_write.err; exit 1; }
cd $R && python3 tools/pmc_sp_summary.py gpurun_out/${1:-r04pmc} gpurun_out/${1:-r04pmc}/pmc_sp_product.json > /dev/null && echo pmc ok
