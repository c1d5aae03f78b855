#!/bin/bash
# round 4 same-box A/B of the C2 bench line: env settings given as arguments ("" = default), each
# run twice, interleaved
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r04ab}
mkdir -p $OUT
cd $R
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/ab_$i.json 2> $OUT/ab_$i.err || { echo "run $i ($e) failed"; tail -5 $OUT/ab_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/ab_$i.json'));r=d['roofline'];print('[$e]', d['config'].get('pcg_continuations_per_trial'), round(d['value'],1), round(d['ms_per_step'],4), r['phase1']['us'], r['phase2']['us'], r['cg_iteration_us'], d['config']['trials_per_iteration'], d['config']['cg_iterations_per_pcg_trial'], d['trial_kernel_ms'].get('sp_glin_rows'), d['trial_kernel_ms'].get('lin_arap'))"
  done
done
