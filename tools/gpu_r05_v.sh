#!/bin/bash
# r05 call V: k_bn_miller_l (two waves, the line / new.y / v0 in LDS) - correctness, then timing alone
# (k = 4 / 2) and pipelined at 65,536 checks against the one-wave k_bn_miller
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05v; mkdir -p $O
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_bn256.py -k "two_wave or rank_batch or random_batch" > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SWEEP_CASES="4,,0;2,,0" $T 300 python -u tools/pairing_sweep.py 65536 > $O/alone_base.txt 2>&1 && grep checks $O/alone_base.txt && \
GSV_BN_MILLER_L=1 SWEEP_CASES="4,,0;2,,0" $T 300 python -u tools/pairing_sweep.py 65536 > $O/alone_ml.txt 2>&1 && sed 's/^/ml /' $O/alone_ml.txt | grep checks && \
GSV_BN_MILLER_L=1 SWEEP_PIPELINE="1,2,3,1,2" $T 300 python -u tools/pairing_sweep.py 65536 8192 > $O/pipe_ml.txt 2>&1 && sed 's/^/ml /' $O/pipe_ml.txt | grep checks && \
SWEEP_PIPELINE="1,2,1,2" $T 300 python -u tools/pairing_sweep.py 65536 > $O/pipe_base.txt 2>&1 && grep checks $O/pipe_base.txt
