#!/bin/bash
# r05 call AD: the large ecrecover differential test (131,072 signatures vs the oracle restatement)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_secp256k1.py > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|passed|failed|Error" $O/tests.log | tail -15; exit $rc
