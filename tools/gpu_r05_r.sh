#!/bin/bash
# r05 call R: chunk-root and notary pipeline depth on dedicated-queue streams, then the default bench
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05r; mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do
  for d in 1 2 3; do
    $T 300 python bench.py --legs chunk_root,notary --pipeline $d --notary-pipeline $d --no-cpu-baseline > $O/cn_d${d}_$rep.json 2> $O/cn_d${d}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/cn_d${d}_$rep.json')); print('depth $d rep $rep: chunk', d['collation_GBps'], 'GB/s', d['chunk_root']['ms_per_step'], 'ms | notary', d['notary']['shards_per_s'], d['notary']['ms_per_step'], 'ms')"
  done
done
$T 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && python3 -c "
import json; d=json.load(open('$O/bench_default.json')); print('default bench', d['value'], d['collation_GBps'], d['bn256_pairing']['checks_per_s'], d['bn256_pairing']['pipeline_depth'], d['notary']['shards_per_s'])"
