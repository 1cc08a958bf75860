#!/bin/bash
# r05 call AG: GPU tests after the side-stream init change (full suite)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; exit $rc
