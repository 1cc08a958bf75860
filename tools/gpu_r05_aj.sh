#!/bin/bash
# r05 call AJ: the fused top at wave priority 3 (GSV_TOP_PRIO=1) now that it runs beside the next
# batch's bottom level for longer (tail mark after the bottom level), against priority 0
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05aj; mkdir -p $O
T="timeout -k 10"
for rep in 1 2 3; do
  for p in 0 1; do
    GSV_TOP_PRIO=$p $T 300 python bench.py --legs chunk_root,notary --no-cpu-baseline > $O/prio${p}_$rep.json 2> $O/prio${p}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/prio${p}_$rep.json')); print('prio $p rep $rep: chunk', d['collation_GBps'], 'GB/s | notary', d['notary']['shards_per_s'])"
  done
done
