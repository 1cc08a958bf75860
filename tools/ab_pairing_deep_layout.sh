#!/bin/bash
# The N = 8 rank batch (8,192 checks) six deep on dedicated-queue streams: the deep rule's layout (k = 4,
# one-lane final, one-wave lines) against the two-wave lines kernel and the three-lane final at the same
# depth, interleaved twice.  GPU box, repo root.
set -o pipefail
O=gpurun_out/ab_pdl; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for L in "auto" "GSV_BN_LINES_W2=1" "GSV_BN_FINAL3=1" "GSV_BN_LINES_W2=1 GSV_BN_FINAL3=1"; do
    if [ "$L" = auto ]; then E=""; else E="$L SWEEP_KEEP_LAYOUT=1"; fi
    T=$(echo "$L" | tr ' =' '__')
    env $E SWEEP_STEPS=36 SWEEP_PIPELINE=6 timeout -k 10 300 python3 tools/pairing_sweep.py 8192 > $O/${T}_r$rep.txt 2>&1 || { echo "$T failed"; tail $O/${T}_r$rep.txt; exit 1; }
    echo "$L: $(grep checks $O/${T}_r$rep.txt)"
  done
done
