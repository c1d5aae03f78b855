#!/bin/bash
# round 3, multi-keyframe workloads on one GPU: smoke, C3 (full, CPU sample), C5 (full, CPU sample),
# C4 (full size)
set -o pipefail
OUT=gpurun_out/${1:-r03m}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
[ -n "$NO_SMOKE" ] || timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
[ -n "$NO_SMOKE" ] || tail -1 $OUT/smoke.log
[ -n "$NO_C3" ] || timeout -k 10 500 python -u bench.py --workload c3 --steps 10 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo c3 failed; tail -20 $OUT/bench_c3.err; exit 1; }
[ -n "$NO_C3" ] || python -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('C3', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'], d['cpu_baseline']['value'])"
timeout -k 10 600 python -u bench.py --workload c5 --steps 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'], d['cpu_baseline']['value'])"
timeout -k 10 700 python -u bench.py --workload c4 --steps 5 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo c4 failed; tail -20 $OUT/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c4.json'));print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'])"
