set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_TILE_PLAIN=1 DEFTRI_SP_TILE_NO_FUSE=1 > gpurun_out/r05h/ab100k.log 2>&1
