#!/bin/bash
# A/B of the ecrecover leg: base library and variants/<name>/libgsv.so given as arguments (secp tests
# against the oracle first, then 3 bench runs each).  Run on the GPU box from the repo root.
set -o pipefail
mkdir -p gpurun_out/abe
for v in base "$@"; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_secp256k1.py -x -q --timeout 120 \
      --timeout-method thread > gpurun_out/abe/test_$v.log 2>&1 || { echo "$v tests failed"; exit 1; }
  for i in 1 2 3; do
    GSV_LIB_PATH=$L timeout -k 10 200 python bench.py --legs ecrecover --no-cpu-baseline --steps 20 \
        > gpurun_out/abe/bench_$v.log 2>&1 || exit 1
    tail -1 gpurun_out/abe/bench_$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" | tee -a gpurun_out/abe/summary.txt || exit 1
  done
done
