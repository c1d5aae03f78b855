set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_GLIN_GROUP=1 > gpurun_out/r05x/ab100k.log 2>&1 && \
timeout -k 10 1300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05x/pytest.log 2>&1
