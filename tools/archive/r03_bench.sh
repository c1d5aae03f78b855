#!/bin/bash
# round-3 GPU pass: smoke, C2 headline, C3 full size and a C4 slice on the iterative plan
set -o pipefail
OUT=gpurun_out/${1:-r03c}
mkdir -p $OUT
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2.json'));print('C2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'])"
timeout -k 10 400 python -u bench.py --workload c3 --steps 10 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo c3 failed; tail -20 $OUT/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'], d['config']['pcg_failed_or_fallback'])"
timeout -k 10 400 python -u bench.py --workload c4 --corr 100000 --steps 5 --no-cpu-baseline > $OUT/bench_c4s.json 2> $OUT/bench_c4s.err || { echo c4 failed; tail -20 $OUT/bench_c4s.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c4s.json'));print('C4 slice', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'])"
