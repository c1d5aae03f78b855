set -o pipefail
mkdir -p gpurun_out/r05ze
export DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py -k "sharded or rccl or tile" tests/test_dist_gpu.py > gpurun_out/r05ze/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/tile_ab.py 100000 10 - > gpurun_out/r05ze/ab.log 2>&1 && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05ze/tile.json 2> gpurun_out/r05ze/tile.err && \
DEFTRI_SP_TXB_KERNEL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29632 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05ze/txbk.json 2> gpurun_out/r05ze/txbk.err
