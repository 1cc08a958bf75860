#!/bin/bash
# r05 call W: the RCCL partition call pipelined on dedicated-queue streams (one-rank communicator) and
# the stream-contract tests
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 160 --timeout-method thread -m gpu tests/test_gpu_partition.py tests/test_gpu_stream_contract.py > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" $O/tests.log | tail -25; exit $rc
