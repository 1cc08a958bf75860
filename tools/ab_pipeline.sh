#!/bin/bash
# A/B of the pipeline depth (shape instances over streams) of the chunk-root and pairing legs.
# Run on the GPU box from the repo root: bash tools/ab_pipeline.sh [depth ...]
set -o pipefail
mkdir -p gpurun_out/p
for d in "${@:-1 2 3}"; do
  timeout -k 10 200 python bench.py --legs chunk_root,pairing --no-cpu-baseline --steps 40 --pipeline $d \
      --pairing-pipeline $d > gpurun_out/p/bench_d$d.log 2>&1 || exit 1
  tail -1 gpurun_out/p/bench_d$d.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); c = d['chunk_root']; p = d['bn256_pairing']
print('depth $d', 'chunk', c['collation_GBps'], 'GB/s', c['ms_per_step'], 'ms', 'pairing', p['checks_per_s'], '/s', p['ms_per_step'], 'ms')" \
      | tee -a gpurun_out/p/summary.txt || exit 1
done
