#!/bin/bash
# r05 call S: deeper pairing pipelines now that each stream has a hardware queue of its own (the r03/r04
# "four queues" ceiling was measured on shared-queue streams): 8,192 and 16,384 checks at depth 4-8,
# auto layout and forced k
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05s; mkdir -p $O
T="timeout -k 10"
SWEEP_PIPELINE="4,5,6,8,4" $T 400 python -u tools/pairing_sweep.py 8192 16384 > $O/deep_auto.txt 2>&1 && grep checks $O/deep_auto.txt && \
GSV_BN_PAIRS_PER_LANE=4 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="4,6,8" $T 300 python -u tools/pairing_sweep.py 8192 > $O/deep_k4.txt 2>&1 && sed 's/^/k4 /' $O/deep_k4.txt | grep checks && \
GSV_BN_PAIRS_PER_LANE=1 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="4,6,8" $T 300 python -u tools/pairing_sweep.py 8192 > $O/deep_k1.txt 2>&1 && sed 's/^/k1 /' $O/deep_k1.txt | grep checks && \
GSV_BN_FINAL3=0 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE="4,6,8" $T 300 python -u tools/pairing_sweep.py 8192 > $O/deep_f1.txt 2>&1 && sed 's/^/final1 /' $O/deep_f1.txt | grep checks
