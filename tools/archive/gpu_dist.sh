#!/bin/bash
# Point-sharded ARAP on one GPU box: the sharded GPU tests (ranks share the GPU through the gloo host
# transport), a 2-rank sharded C2 bench rehearsal (gloo), then an RCCL probe with 2 ranks on one GPU.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-dist}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || { tail -60 $OUT/pytest_dist.log; exit 1; }
tail -5 $OUT/pytest_dist.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline --steps 5 > $OUT/bench1.json 2> $OUT/bench1.err
cat $OUT/bench1.json
DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 > $OUT/bench2_gloo.json 2> $OUT/bench2_gloo.err || { tail -40 $OUT/bench2_gloo.err; exit 1; }
cat $OUT/bench2_gloo.json
timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/probe_rccl.py > $OUT/probe_rccl.log 2>&1 || { tail -30 $OUT/probe_rccl.log; exit 0; }
grep "rank" $OUT/probe_rccl.log | tail -5
