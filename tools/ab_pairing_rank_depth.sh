#!/bin/bash
# The N = 8 rank batch (8,192 checks) by layout and pipeline depth on dedicated-queue streams: auto,
# k = 4 / k = 2 with the one-lane final and no two-lane Miller, at depths 4, 6, 8.  Every Miller / final
# wave holds a SIMD alone (one-wave register budgets), so a k = 4 batch (128 Miller waves) needs about
# eight batches in flight to give every SIMD one.  GPU box, repo root.
set -o pipefail
O=gpurun_out/ab_prd; mkdir -p $O
export PYTHONUNBUFFERED=1
for L in auto "4 0 0" "2 0 0"; do
  set -- $L
  if [ "$1" = auto ]; then E=""; T=auto; else E="GSV_BN_PAIRS_PER_LANE=$1 GSV_BN_FINAL3=$2 GSV_BN_MILLER2=$3 SWEEP_KEEP_LAYOUT=1"; T="k$1f$2m$3"; fi
  env $E SWEEP_STEPS=${STEPS:-48} SWEEP_PIPELINE=${DEPTHS:-4,6,8} timeout -k 10 300 python3 tools/pairing_sweep.py ${CHECKS:-8192} > $O/$T.txt 2>&1 || { echo "$T failed"; tail $O/$T.txt; exit 1; }
  echo "== $T"; grep checks $O/$T.txt
done
