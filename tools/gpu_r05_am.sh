#!/bin/bash
# r05 call AM: the default bench with the pipelined ecrecover leg (two dedicated-queue streams, timing
# events off in the timed region), twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05am; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$rep.json')); r=d['roofline']; print('rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s ms/step', d['ms_per_step'], 'kernel', r['kernel_avg_ms'], 'frac', r['frac'], '| chunk', d['collation_GBps'])"
done
