#!/bin/bash
# r05 call AZ: k_ecrecover ablations (timing only, results wrong by construction): without the comb's
# 12 adds (nocomb), without the final exponentiation (noexp), without r^-1 (noinv), vs in-tree; twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05az; mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do
  $T 120 python -u tools/ecr_time.py main >> $O/t.txt 2>&1 || exit 1
  for v in nocomb noexp noinv; do
    GSV_LIB_PATH=variants/$v/libgsv.so $T 120 python -u tools/ecr_time.py $v >> $O/t.txt 2>&1 || exit 1
  done
done
grep recoveries $O/t.txt
