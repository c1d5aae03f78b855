set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 400 python -u tools/tile_ab.py 100000 25 - DEFTRI_SP_GUESS_HISTORY=0 - DEFTRI_SP_GUESS_HISTORY=0 > gpurun_out/r05z/ab.log 2>&1 && \
DEFTRI_SP_NO_MERGE=1 timeout -k 10 300 python -u tools/tile_ab.py 30000 25 - DEFTRI_SP_GUESS_HISTORY=0 > gpurun_out/r05z/ab30k.log 2>&1
