#!/bin/bash
# round 4: final-exponentiation machine (no private segment) -- GPU tests, then new/base timing
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py tests/test_gpu_partition.py -k "pairing or g2 or synth or precompile or configs4 or partition or ranks" -x -v --timeout 400 --timeout-method thread > gpurun_out/g1_tests.log 2>&1 || { tail -40 gpurun_out/g1_tests.log; exit 1; }
tail -3 gpurun_out/g1_tests.log
SWEEP_CASES="0,,;0,0,;0,1," timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_sweep_new.txt 2>&1 && cat gpurun_out/g1_sweep_new.txt || exit 1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_CASES="0,,;0,0,;0,1," timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_sweep_base.txt 2>&1 && cat gpurun_out/g1_sweep_base.txt || exit 1
SWEEP_PIPELINE=2,3 timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_pipe_new.txt 2>&1 && cat gpurun_out/g1_pipe_new.txt || exit 1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_PIPELINE=2,3 timeout -k 10 300 python tools/pairing_sweep.py 65536 8192 > gpurun_out/g1_pipe_base.txt 2>&1 && cat gpurun_out/g1_pipe_base.txt
