#!/bin/bash
# A/B of the width-4 window exponentiation by u in the final exponentiation (BN_EXPU_W4, main) against
# the NAF chain (variants/now4): pairing GPU tests, the bench's pairing leg alternating, then both
# libraries' per-kernel breakdown at 8,192 / 16,384 checks.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abexpu
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ARGS="--steps 12" timeout -k 10 600 python tools/ab_variants.py pairing main now4 main now4 | tee $O/pairing.txt || exit 1
for v in main now4; do
  if [ $v = main ]; then L=""; else L="variants/$v/libgsv.so"; fi
  echo "$v"
  GSV_LIB_PATH=$L SWEEP_CASES=",," timeout -k 10 300 python tools/pairing_sweep.py 8192 16384 > $O/bd_$v.txt 2>&1 || { tail $O/bd_$v.txt; exit 1; }
  grep checks $O/bd_$v.txt
  GSV_LIB_PATH=$L SWEEP_PIPELINE=2 timeout -k 10 300 python tools/pairing_sweep.py 8192 > $O/pipe_$v.txt 2>&1 || { tail $O/pipe_$v.txt; exit 1; }
  grep checks $O/pipe_$v.txt
done
