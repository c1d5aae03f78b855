set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05g
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05g/fused -o run -- python3 -u tools/tile_ab.py --one 100000 10 > gpurun_out/r05g/fused.log 2>&1 && \
DEFTRI_SP_TILE_NO_FUSE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r05g/unfused -o run -- python3 -u tools/tile_ab.py --one 100000 10 > gpurun_out/r05g/unfused.log 2>&1
