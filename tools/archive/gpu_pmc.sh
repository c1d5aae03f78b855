#!/bin/bash
# HBM traffic counters for the bench's kernels: FETCH_SIZE and WRITE_SIZE in separate rocprofv3
# passes (they do not fit one TCC pass), kernel trace only — no other trace domains with --pmc.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.json 2> $OUT/fetch.err
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.json 2> $OUT/write.err
ls $OUT/fetch $OUT/write
