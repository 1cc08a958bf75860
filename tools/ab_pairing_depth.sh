#!/bin/bash
# Pairing throughput against pipeline depth with the depth-aware layout choice (bn_pairs_per_lane /
# bn_miller2 at depth >= 3): auto layouts at depths 2-4 for the per-rank batches of N = 8, 4, 2, 1,
# then the bench's pairing leg at --pairing-pipeline 2 / 3 / 4.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abdepth
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn256.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SWEEP_PIPELINE=2,3,4 timeout -k 10 500 python tools/pairing_sweep.py 8192 16384 32768 65536 > $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
grep checks $O/sweep.txt
for d in 2 3 4; do
  AB_ARGS="--steps 12 --pairing-pipeline $d" timeout -k 10 300 python tools/ab_variants.py pairing main | sed "s/^/depth $d: /" || exit 1
done
