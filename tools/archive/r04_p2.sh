set -o pipefail
mkdir -p gpurun_out/r04p2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sp.py -k "step_size" > gpurun_out/r04p2/pytest.log 2>&1 || { tail -30 gpurun_out/r04p2/pytest.log; exit 1; }
tail -3 gpurun_out/r04p2/pytest.log
TAG=r04p2 bash tools/r04_ab.sh "" "DEFTRI_SP_ROW_SPLIT=1 DEFTRI_SP_P2_STEP=8" "DEFTRI_SP_ROW_SPLIT=1" "DEFTRI_SP_ROW_SPLIT=4" "DEFTRI_SP_P2_STEP=8"
