#!/bin/bash
# round 4: final exponentiation with width-4 digits (odd powers in the workspace, fetched into LDS by
# global_load_lds) -- GPU tests, then interleaved A/B against the NAF build and the r03 library
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py -k "pairing or g2 or synth or precompile or configs4" -x -v --timeout 400 --timeout-method thread > gpurun_out/g2_tests.log 2>&1 || { tail -40 gpurun_out/g2_tests.log; exit 1; }
tail -2 gpurun_out/g2_tests.log
for rep in 1 2; do
  for lib in new fe_naf base_r03; do
    if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
    echo "== $lib rep $rep"
    env $L SWEEP_CASES="0,," timeout -k 10 200 python tools/pairing_sweep.py 65536 8192 2>&1 | grep checks || exit 1
    env $L SWEEP_PIPELINE=2,3 timeout -k 10 200 python tools/pairing_sweep.py 65536 8192 2>&1 | grep checks || exit 1
  done
done
bash tools/ab_pairing_hwq.sh > gpurun_out/g2_hwq.txt 2>&1; echo "hwq sweep rc=$?"; grep -E "queues|checks" gpurun_out/g2_hwq.txt | head -60
