#!/bin/bash
# r05 call P: pairing pipeline depth on dedicated-queue streams, by batch size
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05p; mkdir -p $O
T="timeout -k 10"
SWEEP_PIPELINE="1,2,3,4,1,2" $T 600 python -u tools/pairing_sweep.py 65536 32768 16384 8192 > $O/depth_own.txt 2>&1 && grep checks $O/depth_own.txt && \
SWEEP_TORCH_STREAMS=1 SWEEP_PIPELINE="1,2,3,1,2" $T 300 python -u tools/pairing_sweep.py 65536 > $O/depth_torch.txt 2>&1 && grep checks $O/depth_torch.txt
