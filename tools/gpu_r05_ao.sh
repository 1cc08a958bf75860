#!/bin/bash
# r05 call AO: the default bench (20 steps after 4 warm-up, pipelined ecrecover leg) twice, with the
# standalone stream A/B on the same box
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ao; mkdir -p $O
timeout -k 10 300 python -u tools/ecr_streams_ab.py > $O/script.txt 2>&1 && grep rep $O/script.txt | tail -1
for rep in 1 2; do
  t0=$(date +%s); timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || exit 1
  echo "bench wall $(( $(date +%s) - t0 )) s"
  python3 -c "
import json; d=json.load(open('$O/bench_$rep.json')); r=d['roofline']; print('rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s ms/step', d['ms_per_step'], 'kernel', r['kernel_avg_ms'], 'frac', r['frac'], '| chunk', d['collation_GBps'], '| pairing', d['bn256_pairing']['checks_per_s'], '| notary', d['notary']['shards_per_s'])"
done
