set -o pipefail
mkdir -p gpurun_out/r05zc
export DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_sp.py -k "sharded_iterative_matches_oracle" > gpurun_out/r05zc/pytest.log 2>&1 && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05zc/tile.json 2> gpurun_out/r05zc/tile.err && \
DEFTRI_SP_SD_NO_TILE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29622 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05zc/notile.json 2> gpurun_out/r05zc/notile.err
