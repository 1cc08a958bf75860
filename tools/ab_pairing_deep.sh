#!/bin/bash
# Pairing at the N = 8 per-rank batch (8,192 checks) with 4-8 batches in flight under forced layouts.  GPU box.
set -o pipefail
for lay in "auto" "4 0 0" "2 0 0" "2 1 0"; do
  set -- $lay
  if [ "$1" = auto ]; then E=""; else E="GSV_BN_PAIRS_PER_LANE=$1 GSV_BN_FINAL3=$2 GSV_BN_MILLER2=$3"; fi
  echo "layout k/final3/miller2 = $lay"
  env $E SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE=4,6,8 timeout -k 10 300 python tools/pairing_sweep.py 8192 > gpurun_out/lp2_${1}${2}${3}.txt 2>&1 || { tail gpurun_out/lp2_${1}${2}${3}.txt; exit 1; }
  grep checks gpurun_out/lp2_${1}${2}${3}.txt
done
