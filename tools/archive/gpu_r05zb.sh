set -o pipefail
mkdir -p gpurun_out/r05zb
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py -k "sharded or rccl" tests/test_dist_gpu.py > gpurun_out/r05zb/pytest.log 2>&1
