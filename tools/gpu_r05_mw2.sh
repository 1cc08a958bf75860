#!/bin/bash
# r05: Miller kernel at a two-wave register budget (variants/mw2, spilling) vs the one-wave build,
# at the configs[4] batch with k = 4 / 2 pairs per Miller lane and the N = 8 batch pipelined
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r05
for v in base mw2; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L SWEEP_CASES="4,,;2,,;1,," timeout -k 10 240 python -u tools/pairing_sweep.py 65536 \
      > gpurun_out/r05/mw2_sweep_$v.txt 2>&1 || { echo "$v failed"; cat gpurun_out/r05/mw2_sweep_$v.txt; exit 1; }
  GSV_LIB_PATH=$L SWEEP_PIPELINE="2,3" timeout -k 10 240 python -u tools/pairing_sweep.py 65536 8192 \
      >> gpurun_out/r05/mw2_sweep_$v.txt 2>&1 || { echo "$v pipe failed"; cat gpurun_out/r05/mw2_sweep_$v.txt; exit 1; }
  sed "s/^/$v /" gpurun_out/r05/mw2_sweep_$v.txt
done
