#!/bin/bash
# Pipelined throughput of small pairing batches (the per-rank batch at N = 4 / 8) under forced layouts:
# work-efficient (4 pairs per Miller lane, one-lane final) against latency-oriented (1 pair per lane,
# two-lane Miller, three-lane final), at pipeline depths 2-4.  GPU box, repo root.
set -o pipefail
O=gpurun_out/ablp
mkdir -p $O
for lay in "auto" "4 0 0" "2 0 0" "4 1 0" "2 1 0" "1 1 1" "1 0 1"; do
  set -- $lay
  if [ "$1" = auto ]; then E=""; else E="GSV_BN_PAIRS_PER_LANE=$1 GSV_BN_FINAL3=$2 GSV_BN_MILLER2=$3"; fi
  echo "layout k/final3/miller2 = $lay"
  env $E SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE=2,3,4 timeout -k 10 300 python tools/pairing_sweep.py 8192 16384 > $O/lay_${1}${2}${3}.txt 2>&1 || { tail $O/lay_${1}${2}${3}.txt; exit 1; }
  grep checks $O/lay_${1}${2}${3}.txt
done
