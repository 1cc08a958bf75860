#!/bin/bash
# A/B of pairing-kernel variants at the configs[4] batch and the N = 8 per-rank batch: base library
# and variants/<name>/libgsv.so given as arguments (tools/pairing_sweep.py at auto layout, depth 1).
set -o pipefail
mkdir -p gpurun_out/abp
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L SWEEP_CASES="0,," timeout -k 10 200 python -u tools/pairing_sweep.py 65536 8192 \
      > gpurun_out/abp/sweep_$v.txt 2>&1 || { echo "$v failed"; exit 1; }
  grep checks gpurun_out/abp/sweep_$v.txt | sed "s/^/$v /" | tee -a gpurun_out/abp/summary.txt
done
