#!/bin/bash
# r05 call AV: Keccak leg workload (400 k tx strings) by workgroup size (GSV_KECCAK_BLOCK), twice interleaved
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05av; mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do for b in 256 128 64; do
  GSV_KECCAK_BLOCK=$b $T 120 python -u tools/keccak_sweep.py block$b > $O/b${b}_$rep.txt 2>&1 || exit 1
  grep depth $O/b${b}_$rep.txt
done; done
