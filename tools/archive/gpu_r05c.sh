set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 300 python -u tools/tile_ab.py 20000 5 > gpurun_out/r05c/ab20k.log 2>&1 && \
timeout -k 10 600 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_NO_TILE=1 DEFTRI_SP_TILE_LDS=39500 DEFTRI_SP_TILE_UNITS=64 > gpurun_out/r05c/ab100k.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py::test_native_outer_loop_matches_host_loop tests/test_gpu_parity.py::test_weight_search_matches_oracle tests/test_c2_golden.py tests/test_full_size_props.py::test_c2_full_size_properties > gpurun_out/r05c/pytest.log 2>&1
