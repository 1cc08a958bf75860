#!/bin/bash
# r05 call AW: Keccak leg workload, batches in flight 1-4 (dedicated queues), twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05aw; mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do
  KECCAK_DEPTHS=1,2,3,4 $T 120 python -u tools/keccak_sweep.py depth > $O/d_$rep.txt 2>&1 || exit 1
  grep depth $O/d_$rep.txt
done
