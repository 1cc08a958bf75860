#!/bin/bash
# r05 call AQ: the ecrecover leg on one stream with events over the timed region (default) vs two
# streams with a separate instrumented pass, same box, 3 x interleaved; then the leg-only trace pass
# with per-dispatch durations (same-launch trace agreement)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05aq; mkdir -p $O
for rep in 1 2 3; do
  for d in 1 2; do
    timeout -k 10 300 python bench.py --legs ecrecover --no-cpu-baseline --ecrecover-pipeline $d > $O/e${d}_$rep.json 2> $O/e${d}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/e${d}_$rep.json')); r=d['roofline']; print('depth $d rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s ms/step', d['ms_per_step'], 'kernel', r['kernel_avg_ms'], 'launches', r['kernel_launches_timed'], 'frac', r['frac'])"
  done
done
