set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05y; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 bench.py --steps 25 --warmup 3 --no-legs --no-e2e --no-cpu-baseline --trace-markers > $OUT/tr.json 2> $OUT/tr.err && \
DEFTRI_CALL_TIMING=1 DEFTRI_PLAN_TIMING=1 DEFTRI_UPLOAD_TIMING=1 DEFTRI_GRAPH_TIMING=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-legs --no-cpu-baseline > $OUT/e2e.json 2> $OUT/e2e.err
