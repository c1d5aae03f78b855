set -o pipefail
mkdir -p gpurun_out/r05u
export DEFTRI_DIST_BACKEND=gloo DEFTRI_GPU_OVERRIDE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05u/rehearsal_ovl.json 2> gpurun_out/r05u/rehearsal_ovl.err && \
DEFTRI_SP_NO_OVERLAP=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 10 --warmup 2 --no-legs --no-e2e --no-cpu-baseline > gpurun_out/r05u/rehearsal_serial.json 2> gpurun_out/r05u/rehearsal_serial.err
