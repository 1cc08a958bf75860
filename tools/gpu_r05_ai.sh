#!/bin/bash
# r05 call AI: the notary's per-rank shares at N = 8 / 4 (13 / 25 shards) deeper in flight (depth 2-6)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ai; mkdir -p $O
NOTARY_DEPTHS="2,3,4,5,6,3" timeout -k 10 500 python -u tools/notary_sweep.py 13 25 > $O/notary_deep.txt 2>&1 && grep shards $O/notary_deep.txt
