set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_TILE_TICKETS=1 DEFTRI_SP_NO_TILE=1 > gpurun_out/r05j/ab100k.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_full_size_props.py::test_c2_full_size_properties tests/test_c2_golden.py tests/test_regime_goldens.py tests/test_gpu_sp.py -k "not sharded and not rccl" > gpurun_out/r05j/pytest.log 2>&1
