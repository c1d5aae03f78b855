#!/bin/bash
# round 3: C3 / C4 / C5 on the current build (merged CG chain), no CPU baselines (their samples are in r03h_bench_c{3,5}.json)
set -o pipefail
OUT=gpurun_out/${1:-r03t}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for w in c3 c5 c4; do
  timeout -k 10 500 python -u bench.py --workload $w --steps ${2:-5} --no-cpu-baseline --no-e2e > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo $w failed; tail -20 $OUT/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$w.json'));r=d['roofline'];c=d['config'];print('$w', round(d['value'],2), round(d['ms_per_step'],1), r['frac'], r['cg_iteration_us'], r['phase1']['us'], r['phase2']['us'], c.get('cg_iterations_per_pcg_trial'), c.get('pcg_failed_or_fallback'))"
done
