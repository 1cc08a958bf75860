#!/bin/bash
# r05 call U: notary per-rank shares (100 / 50 / 25 / 13 shards) on dedicated-queue streams, depth 1-3
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 500 python -u tools/notary_sweep.py 100 50 25 13 > $O/notary_shares.txt 2>&1 && grep shards $O/notary_shares.txt
