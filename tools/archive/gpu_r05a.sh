set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py::test_alpha_hand_off_timeout_is_an_error tests/test_full_size_props.py::test_c5_full_size_properties -s > gpurun_out/r05a/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err
