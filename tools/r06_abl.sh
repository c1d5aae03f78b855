#!/bin/bash
# round 6: kernel times of build variants (ab/libdeftri_*.so) at C2 under rocprofv3 --kernel-trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06abl}
N=${2:-100000}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in $R/ab/libdeftri_*.so; do
  v=$(basename $lib .so)
  DEFTRI_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python3 $R/tools/abl_run.py $N 4 > $OUT/$v.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v.log; exit 1; }
  echo "$v $(python3 $R/tools/abl_run.py --summ $OUT/$v)"
done
