#!/bin/bash
# r05 call AY: upper bound of removing r^-1 mod n from k_ecrecover (variants/noinv: timing only, wrong
# results by construction) against the in-tree library, interleaved twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ay; mkdir -p $O
T="timeout -k 10"
for rep in 1 2; do
  $T 120 python -u tools/ecr_time.py main >> $O/t.txt 2>&1 || exit 1
  GSV_LIB_PATH=variants/noinv/libgsv.so $T 120 python -u tools/ecr_time.py noinv >> $O/t.txt 2>&1 || exit 1
done
grep recoveries $O/t.txt
