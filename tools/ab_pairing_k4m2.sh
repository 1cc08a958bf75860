#!/bin/bash
# Small pairing batches at depth 3-4: k = 4 / 2 pairs per Miller lane with the two-lane Miller step (more waves per launch at four-pairs-per-lane work) against the auto layout.  GPU box.
set -o pipefail
for lay in "auto" "4 1 1" "2 1 1" "2 1 0"; do
  set -- $lay
  if [ "$1" = auto ]; then E=""; else E="GSV_BN_PAIRS_PER_LANE=$1 GSV_BN_FINAL3=$2 GSV_BN_MILLER2=$3"; fi
  echo "layout k/final3/miller2 = $lay"
  env $E SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE=3,4 timeout -k 10 300 python tools/pairing_sweep.py 8192 16384 > gpurun_out/lp3_${1}${2}${3}.txt 2>&1 || { tail gpurun_out/lp3_${1}${2}${3}.txt; exit 1; }
  grep checks gpurun_out/lp3_${1}${2}${3}.txt
done
