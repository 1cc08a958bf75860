#!/bin/bash
# r05 call E: the pairing pipeline with both two-wave kernels (lines and Miller: 256 + 256 registers can
# share a SIMD, so batch B's lines run beside batch A's Miller loop), against lines-only two-wave and
# the one-wave pair, at the configs[4] batch (depth 2, 3) and the N = 8 rank batch (depth 3, 4)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05e; mkdir -p $O
T="timeout -k 10"
for cfg in "1 1" "1 0" "0 0" "0 1"; do
  set -- $cfg
  for n in 65536 8192; do
    if [ $n = 65536 ]; then D="2,3,2,3"; else D="3,4,3,4"; fi
    GSV_BN_LINES_W2=$1 GSV_BN_MILLER_W2=$2 SWEEP_PIPELINE=$D $T 300 python -u tools/pairing_sweep.py $n > $O/pipe_l$1_m$2_$n.txt 2>&1 || { echo pipe $cfg $n failed; tail $O/pipe_l$1_m$2_$n.txt; exit 1; }
    grep checks $O/pipe_l$1_m$2_$n.txt | sed "s/^/lines_w2=$1 miller_w2=$2 /"
  done
done
