#!/bin/bash
# A/B of the concurrent-check pairing layout (GSV_BN_LAYOUT_CONC): the pairing GPU tests (which run
# small batches, i.e. the concurrent path, incl. bad inputs, points outside G2 and graph capture), then
# pipelined sweeps with the layout forced off / on.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abconc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in 0 1; do
  GSV_BN_CONC=$c SWEEP_PIPELINE=1,2,3 timeout -k 10 400 python tools/pairing_sweep.py 8192 16384 65536 > $O/sweep_conc$c.txt 2>&1 || { echo "sweep $c failed"; tail -20 $O/sweep_conc$c.txt; exit 1; }
  echo "GSV_BN_CONC=$c"; cat $O/sweep_conc$c.txt
done
