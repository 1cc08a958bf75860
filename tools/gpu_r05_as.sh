#!/bin/bash
# r05 call AS: chunk-root pipeline depth 2 / 3 / 4 at the 20-step default, interleaved twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05as; mkdir -p $O
for rep in 1 2; do
  for d in 2 3 4; do
    timeout -k 10 300 python bench.py --legs chunk_root --pipeline $d --no-cpu-baseline > $O/c${d}_$rep.json 2> $O/c${d}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/c${d}_$rep.json')); print('depth $d rep $rep: chunk', d['collation_GBps'], 'GB/s', d['chunk_root']['ms_per_step'], 'ms')"
  done
done
