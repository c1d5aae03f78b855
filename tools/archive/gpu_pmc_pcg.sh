#!/bin/bash
# rocprofv3 passes over a short C2 bench run (PCG steps): kernel-trace stats, then one counter set
# per pass (FETCH_SIZE; WRITE_SIZE; TCC hit/miss) — never combined with other trace domains.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-pmcpcg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.json 2> $OUT/fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.json 2> $OUT/write.err
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/tcc -o run -- python3 $B > $OUT/tcc.json 2> $OUT/tcc.err
ls $OUT/trace $OUT/fetch $OUT/write $OUT/tcc
