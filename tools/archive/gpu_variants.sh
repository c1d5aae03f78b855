#!/bin/bash
# A/B of libdeftri build variants (tools/devlib/libdeftri_<v>.so) on the C2 bench (no CPU baseline).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-var}
mkdir -p $OUT
cd $R
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $OUT/base.json 2>/dev/null
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('base', round(d['value'],2), d['trial_kernel_ms']['update'], d['trial_kernel_ms'].get('hchunk'), d['trial_kernel_ms'].get('hfinal'), d['trial_kernel_ms'].get('bchunk'))" $OUT/base.json
for v in $VARIANTS; do
  DEFTRI_LIB=tools/devlib/libdeftri_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline > $OUT/$v.json 2>/dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value'],2), d['trial_kernel_ms']['update'], d['trial_kernel_ms'].get('hchunk'), d['trial_kernel_ms'].get('hfinal'), d['trial_kernel_ms'].get('bchunk'))" $OUT/$v.json $v
done
