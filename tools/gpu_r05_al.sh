#!/bin/bash
# r05 call AL: the Keccak leg over two dedicated-queue streams, 40 timed batches; tx-root leg 20 steps
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05al; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python bench.py --legs keccak,tx_root --no-cpu-baseline > $O/kt_$rep.json 2> $O/kt_$rep.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/kt_$rep.json'))['collation_extras']; k=d['keccak256']; print('rep $rep: keccak', k['GBps'], 'GB/s', k['ms_per_step'], 'ms/step kernel', k['roofline']['kernel_avg_ms'], '| tx_root', d['tx_root']['txs_per_s'], d['tx_root']['ms_per_step'])"
done
