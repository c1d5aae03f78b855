#!/bin/bash
# full-size C4 (500k x 8 keyframes, all 28 pairs) and C5 (Realcolon 20 x 200k, 19 consecutive pairs)
set -o pipefail
OUT=gpurun_out/${1:-r03d}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --workload c4 --steps ${2:-5} --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo c4 failed; tail -20 $OUT/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c4.json'));print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'], d['config']['pcg_failed_or_fallback'])"
timeout -k 10 500 python -u bench.py --workload c5 --steps ${2:-5} --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c5.json'));print('C5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['config']['cg_iterations_per_pcg_trial'], d['config']['pcg_failed_or_fallback'])"
timeout -k 10 300 python -u bench.py --plan iterative --no-cpu-baseline --no-e2e > $OUT/bench_c2_iter.json 2> $OUT/bench_c2_iter.err || { echo c2 iterative failed; tail -20 $OUT/bench_c2_iter.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c2_iter.json'));print('C2 iterative', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['cg_iteration_us'], d['roofline']['phase1'], d['roofline']['phase2'])"
