set -o pipefail
mkdir -p gpurun_out/r05za
timeout -k 10 600 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_TILE_LDS=52224 DEFTRI_SP_TILE_LDS=45056 > gpurun_out/r05za/ab.log 2>&1
