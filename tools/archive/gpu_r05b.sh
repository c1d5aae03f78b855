set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 300 python -u tools/tile_ab.py 20000 5 > gpurun_out/r05b/ab20k.log 2>&1 && \
timeout -k 10 300 python -u tools/tile_ab.py 100000 10 > gpurun_out/r05b/ab100k.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py::test_alpha_hand_off_timeout_is_an_error tests/test_full_size_props.py::test_c5_full_size_properties tests/test_full_size_props.py::test_c2_full_size_properties -s > gpurun_out/r05b/pytest.log 2>&1
