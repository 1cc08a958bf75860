#!/bin/bash
# k_notary_tx per tx against k_ecrecover per recovery: the notary step one at a time with no side streams
# (GSV_MAX_SIDE_STREAMS=0, so the chunk roots run after the transactions and the "tx kernels" time is the
# blob index + k_notary_tx alone) at 100 shards (819,200 txs = 12,800 waves = 6.25 rounds of the GPU's
# 2,048 wave slots at two waves per SIMD) and 128 shards (2^20 txs = 16,384 waves = 8 whole rounds),
# beside the bench's ecrecover leg (2^20 recoveries = 8 whole rounds).  GPU box, repo root.
set -o pipefail
O=gpurun_out/ab_nq; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  GSV_MAX_SIDE_STREAMS=0 NOTARY_DEPTHS=1 NOTARY_STEPS=12 timeout -k 10 300 python3 tools/notary_sweep.py 100 128 64 > $O/notary_r$rep.txt 2>&1 || { echo "sweep failed"; tail $O/notary_r$rep.txt; exit 1; }
  grep shards $O/notary_r$rep.txt
  timeout -k 10 300 python3 bench.py --legs ecrecover --no-cpu-baseline --steps 20 > $O/ecr_r$rep.log 2>&1 || { echo "bench failed"; tail $O/ecr_r$rep.log; exit 1; }
  tail -1 $O/ecr_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ecrecover', d['value'], 'recoveries/s', d['ms_per_step'], 'ms per 2^20, kernel', d['roofline'].get('kernel_avg_ms'))"
done
