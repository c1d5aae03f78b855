set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sp.py::test_tile_linearization_matches_row_gathers > gpurun_out/r05o/pytest0.log 2>&1 && \
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_TILE_GLIN_ROWS=1 > gpurun_out/r05o/ab100k.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_full_size_props.py::test_c2_full_size_properties tests/test_c2_golden.py tests/test_regime_goldens.py tests/test_gpu_sp.py -k "not sharded and not rccl" > gpurun_out/r05o/pytest.log 2>&1
