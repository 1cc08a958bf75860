#!/bin/bash
# r05 call AE: run-to-run spread of the default bench on one box (5 runs, CPU baseline off), to back
# the ranges quoted in README / DESIGN §0 with one box's repeat figures
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ae; mkdir -p $O
for rep in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/bench_$rep.json')); print('rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s | chunk', d['collation_GBps'], 'GB/s | pairing', round(d['bn256_pairing']['checks_per_s']/1e6,3), 'M/s | notary', d['notary']['shards_per_s'], '| keccak', d['collation_extras']['keccak256']['GBps'])"
done
