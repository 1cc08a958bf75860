#!/bin/bash
# The bench's headline leg (configs[1], 2^20 recoveries per batch) at --ecrecover-pipeline 1 / 2 / 3 / 4,
# twice in alternation (run through gpurun from the repo root).
set -o pipefail
O=gpurun_out/ed; mkdir -p $O
for r in 1 2; do
  for d in 1 2 3 4; do
    timeout -k 10 300 python bench.py --legs ecrecover --no-cpu-baseline --ecrecover-pipeline $d --steps 40 > $O/bench_d${d}_$r.log 2>&1 || { echo "depth $d bench failed"; tail -5 $O/bench_d${d}_$r.log; exit 1; }
    tail -1 $O/bench_d${d}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth $d', d['value'], 'recoveries/s', d['ms_per_step'], 'ms/step')"
  done
done
