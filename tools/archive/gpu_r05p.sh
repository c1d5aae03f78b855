set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - > gpurun_out/r05p/ab100k.log 2>&1 && \
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05p/pytest.log 2>&1
