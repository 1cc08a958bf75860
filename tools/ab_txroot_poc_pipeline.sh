#!/bin/bash
# The bench's tx-root and POC legs one batch at a time (--pipeline 1) against two and three batches in
# flight on dedicated-queue streams (2, the default), twice in alternation (run through gpurun from the
# repo root).
set -o pipefail
O=gpurun_out/tp; mkdir -p $O
for r in 1 2; do
  for d in 1 2 3; do
    timeout -k 10 300 python bench.py --legs tx_root,poc --no-cpu-baseline --pipeline $d > $O/bench_d${d}_$r.log 2>&1 || { echo "depth $d bench failed"; tail -5 $O/bench_d${d}_$r.log; exit 1; }
    tail -1 $O/bench_d${d}_$r.log | python3 -c "import json,sys; e=json.loads(sys.stdin.read())['collation_extras']; print('depth $d', 'tx_root', e['tx_root']['txs_per_s'], e['tx_root']['ms_per_step'], 'ms | poc', e['proof_of_custody']['bodies_per_s'], e['proof_of_custody']['ms_per_step'], 'ms')"
  done
done
