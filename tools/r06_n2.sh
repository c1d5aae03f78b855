#!/bin/bash
# round 6: the N > 1 bench line rehearsed with 2 ranks on one GPU (gloo transport), the c4 leg on a
# 50k-per-keyframe slice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06n2}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0 timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --c4-corr 50000 > $OUT/bench2.json 2> $OUT/bench2.err || { tail -40 $OUT/bench2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench2.json')); print(d['metric'], d['value'], d['n_gpus'], d['scaling'], d['config'].get('parallelism')); print('c4', json.dumps(d.get('c4'))[:600]); print('500k', json.dumps(d.get('north_star_500k'))[:400])"
