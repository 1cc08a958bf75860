#!/bin/bash
# A/B of the two-lane line precomputation (GSV_BN_LAYOUT_LINES2, small batches): the pairing GPU tests
# (small batches: the lines2 path, incl. bad inputs and graph capture), then pipelined sweeps with the
# layout forced off / on.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abl2
mkdir -p $O
GSV_BN_LINES2=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 0 1; do
  GSV_BN_LINES2=$c SWEEP_PIPELINE=1,2 timeout -k 10 400 python tools/pairing_sweep.py 8192 4096 16384 > $O/sweep_l2_$c.txt 2>&1 || { echo "sweep $c failed"; tail -20 $O/sweep_l2_$c.txt; exit 1; }
  echo "GSV_BN_LINES2=$c"; cat $O/sweep_l2_$c.txt
done
GSV_BN_LINES2=1 SWEEP_CASES=",,;" timeout -k 10 300 python tools/pairing_sweep.py 8192 16384 > $O/breakdown_l2.txt 2>&1 || exit 1
GSV_BN_LINES2=0 SWEEP_CASES=",,;" timeout -k 10 300 python tools/pairing_sweep.py 8192 16384 > $O/breakdown_l1.txt 2>&1 || exit 1
cat $O/breakdown_l1.txt $O/breakdown_l2.txt
