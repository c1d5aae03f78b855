set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05i
timeout -k 10 400 python -u tools/tile_ab.py 100000 10 - DEFTRI_SP_ALPHA_KERNEL=1 DEFTRI_SP_NO_TILE=1 > gpurun_out/r05i/ab100k.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r05i/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05i/prof -o run -- python3 -u bench.py --steps 10 --warmup 3 --no-legs --no-e2e > gpurun_out/r05i/prof.log 2>&1
