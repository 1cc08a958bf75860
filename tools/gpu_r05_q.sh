#!/bin/bash
# r05 call Q: pairing pipeline depth on dedicated-queue streams (destroyed after each run), by batch size
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05q; mkdir -p $O
T="timeout -k 10"
SWEEP_PIPELINE="1,2,3,4,1,2,3,4" $T 900 python -u tools/pairing_sweep.py 65536 32768 16384 8192 > $O/depth_own.txt 2>&1 && grep checks $O/depth_own.txt
