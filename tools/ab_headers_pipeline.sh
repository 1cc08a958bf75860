#!/bin/bash
# The bench's collation-header leg one batch at a time (--ecrecover-pipeline 1) against two batches in
# flight on dedicated-queue streams (2, the default), twice in alternation (run through gpurun from the
# repo root).
set -o pipefail
O=gpurun_out/hp; mkdir -p $O
for r in 1 2; do
  for d in 1 2; do
    timeout -k 10 300 python bench.py --legs ecrecover,headers --no-cpu-baseline --ecrecover-pipeline $d > $O/bench_d${d}_$r.log 2>&1 || { echo "depth $d bench failed"; tail -5 $O/bench_d${d}_$r.log; exit 1; }
    tail -1 $O/bench_d${d}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['collation_extras']['collation_headers']; print('depth $d', d['headers_per_s'], 'headers/s', d['ms_per_step'], 'ms/step')"
  done
done
