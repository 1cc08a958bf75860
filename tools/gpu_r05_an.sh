#!/bin/bash
# r05 call AN: same-box comparison of the standalone ecrecover stream A/B and the bench's leg
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05an; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u tools/ecr_streams_ab.py > $O/script_$rep.txt 2>&1 || exit 1
  grep rep $O/script_$rep.txt | tail -1
  timeout -k 10 300 python bench.py --legs ecrecover --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$rep.json')); r=d['roofline']; print('bench rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s ms/step', d['ms_per_step'], 'kernel', r['kernel_avg_ms'])"
  timeout -k 10 300 python bench.py --legs ecrecover --no-cpu-baseline --steps 20 --warmup 4 > $O/bench20_$rep.json 2> $O/bench20_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench20_$rep.json')); r=d['roofline']; print('bench steps 20 rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s ms/step', d['ms_per_step'], 'kernel', r['kernel_avg_ms'])"
done
