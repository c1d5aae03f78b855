#!/bin/bash
# regime goldens on the device, C5 precision sweep, 2-rank sharded bench rehearsal (gloo, one GPU)
set -o pipefail
OUT=gpurun_out/${1:-r03i}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_regime_goldens.py -v --timeout 300 --timeout-method thread > $OUT/test_regimes.log 2>&1; echo "regimes rc=$?"; tail -8 $OUT/test_regimes.log
timeout -k 10 300 env DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_sharded2.json 2> $OUT/bench_sharded2.err; echo "sharded rc=$?"; tail -c 1500 $OUT/bench_sharded2.json
timeout -k 10 500 python -u tools/precision_sweep_c5.py $OUT/precision_sweep.json 200000 10 c5w c5a > $OUT/precision.log 2>&1; echo "sweep rc=$?"; tail -4 $OUT/precision.log
