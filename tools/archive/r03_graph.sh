#!/bin/bash
# round 3: graph-build timings (host threads vs device computeR), plan reuse, e2e bench line
set -o pipefail
mkdir -p gpurun_out/r03g
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py tests/test_gpu_sp.py > gpurun_out/r03g/pytest.log 2>&1 &&
for t in 1 4 16; do DEFTRI_HOST_THREADS=$t DEFTRI_NO_GRAPH_MEMO=1 DEFTRI_GRAPH_TIMING=1 timeout -k 10 120 python tools/graph_timing.py 100000 2 --check tools/graph_digest_c2.json >> gpurun_out/r03g/graph_host.log 2>&1 || exit 1; done &&
DEFTRI_NO_GRAPH_MEMO=1 DEFTRI_GRAPH_TIMING=1 timeout -k 10 120 python tools/graph_timing.py 100000 3 --device 0 --check tools/graph_digest_c2.json > gpurun_out/r03g/graph_dev.log 2>&1 &&
DEFTRI_GRAPH_TIMING=1 timeout -k 10 300 python bench.py --steps 25 --warmup 2 > gpurun_out/r03g/bench.json 2> gpurun_out/r03g/bench.err
[ $? -eq 0 ] || exit 1
for v in "fused" "fence DEFTRI_SP_FENCE=1" "unfused DEFTRI_SP_NO_FUSE=1"; do
  set -- $v
  env $2 timeout -k 10 240 python bench.py --steps 25 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r03g/ab_$1.json 2> gpurun_out/r03g/ab_$1.err || exit 1
done
