set -o pipefail
mkdir -p gpurun_out/r05c
timeout -k 10 300 python -u tools/tile_ab.py 20000 5 > gpurun_out/r05c/ab20k.log 2>&1 && \
timeout -k 10 600 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_NO_TILE=1 DEFTRI_SP_TILE_LDS=39500 DEFTRI_SP_TILE_UNITS=64 > gpurun_out/r05c/ab100k.log 2>&1
