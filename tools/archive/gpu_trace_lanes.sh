#!/bin/bash
# rocprofv3 kernel stats of the C2 LM at 1 and 3 speculative lanes (5 iterations after a warm-up).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-tr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for l in ${LANES:-1 3}; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/l$l -o run -- python3 $R/tools/lane_trace.py 100000 $l 5 > $OUT/l$l.txt 2>&1
grep lanes $OUT/l$l.txt
done
