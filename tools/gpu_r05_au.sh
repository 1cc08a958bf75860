#!/bin/bash
# r05 call AU: the N = 8 per-rank pairing batch with the two-wave lines kernel on dedicated queues
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05au; mkdir -p $O
T="timeout -k 10"
GSV_BN_LINES_W2=1 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="3,4,6" $T 300 python -u tools/pairing_sweep.py 8192 > $O/lw2.txt 2>&1 && sed 's/^/lines_w2 /' $O/lw2.txt | grep checks && \
SWEEP_PIPELINE="3,4,6" $T 300 python -u tools/pairing_sweep.py 8192 > $O/auto.txt 2>&1 && sed 's/^/auto /' $O/auto.txt | grep checks
