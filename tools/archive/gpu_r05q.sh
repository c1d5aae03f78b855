set -o pipefail
mkdir -p gpurun_out/r05q
for k in "native_outer" "weight_search_multi or native_outer" "degenerate or native_outer" "minimal or native_outer" "plan_reuse or native_outer"; do
  echo "== $k" >> gpurun_out/r05q/sel.log
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "$k" >> gpurun_out/r05q/sel.log 2>&1
  rc=$?
  if [ $rc -gt 1 ]; then echo "stop rc=$rc" >> gpurun_out/r05q/sel.log; exit $rc; fi
done
