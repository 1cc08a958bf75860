#!/bin/bash
# r05 call AC: the N = 8 per-rank pairing batch (8,192 checks) with the most work-efficient layout
# (k = 4 pairs per Miller lane, one lane per check in the final exponentiation) deeper in flight
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ac; mkdir -p $O
T="timeout -k 10"
GSV_BN_PAIRS_PER_LANE=4 GSV_BN_FINAL3=0 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="4,6,8" $T 300 python -u tools/pairing_sweep.py 8192 > $O/k4f1.txt 2>&1 && sed 's/^/k4 final1 /' $O/k4f1.txt | grep checks && \
GSV_BN_PAIRS_PER_LANE=2 GSV_BN_FINAL3=0 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="4,6,8" $T 300 python -u tools/pairing_sweep.py 8192 > $O/k2f1.txt 2>&1 && sed 's/^/k2 final1 /' $O/k2f1.txt | grep checks && \
SWEEP_PIPELINE="6,8" $T 300 python -u tools/pairing_sweep.py 8192 16384 > $O/auto.txt 2>&1 && sed 's/^/auto /' $O/auto.txt | grep checks
