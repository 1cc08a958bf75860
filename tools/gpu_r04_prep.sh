#!/bin/bash
# pairing: lines tiled by 64-pair group (BN_LINES_TILED) -- parity, then same-bytes A/B against the flat
# layout (variants/lines_flat) and r03
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py -k "pairing or g2 or synth or precompile or configs4" -x -q --timeout 300 --timeout-method thread > gpurun_out/g9_tests.log 2>&1 || { tail -30 gpurun_out/g9_tests.log; exit 1; }
tail -1 gpurun_out/g9_tests.log
bash tools/gpu_r04_miller.sh || exit 1
SWEEP_PIPELINE=2,3 timeout -k 10 200 python tools/pairing_sweep.py 65536 8192 2>&1 | grep checks
