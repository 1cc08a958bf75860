#!/bin/bash
# r05 call AH: k_ecrecover compile options re-measured on the r05 code (GLV table prefetch, all-private
# GLV table, the two digit adds unrolled) against the default; recovery parity under each first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ah; mkdir -p $O
T="timeout -k 10"
for v in pf1 tab1 uj1; do
  GSV_LIB_PATH=variants/$v/libgsv.so $T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_secp256k1.py > $O/tests_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in base pf1 tab1 uj1; do
    if [ $v = base ]; then unset GSV_LIB_PATH; else export GSV_LIB_PATH=variants/$v/libgsv.so; fi
    $T 300 python bench.py --legs ecrecover --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); print('$v rep $rep: ecrecover', round(d['value']/1e6,2), 'M/s kernel', d['roofline']['kernel_avg_ms'], 'ms')"
  done
done
