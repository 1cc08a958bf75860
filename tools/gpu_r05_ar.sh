#!/bin/bash
# r05 call AR: pairing / notary legs with warm-up >= --warmup and >= steps/2 timed batches, twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ar; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --legs notary,pairing --no-cpu-baseline > $O/np_$rep.json 2> $O/np_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/np_$rep.json')); p=d['bn256_pairing']; print('rep $rep: pairing', p['checks_per_s'], p['ms_per_step'], 'ms | notary', d['notary']['shards_per_s'], d['notary']['ms_per_step'])"
done
