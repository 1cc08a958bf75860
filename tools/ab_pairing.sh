#!/bin/bash
# A/B of the pairing leg: the in-tree library and variants/<name>/libgsv.so (pairing GPU tests first),
# then the bench's pairing leg, alternating, 2 runs each.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abpair
mkdir -p $O
for v in main "$@"; do
  if [ $v = main ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_bn256.py -x -q --timeout 160 --timeout-method thread > $O/test_$v.log 2>&1 || { echo "$v tests failed"; exit 1; }
done
AB_ARGS="--steps 12" timeout -k 10 600 python tools/ab_variants.py pairing main "$@" main "$@" | tee $O/summary.txt || exit 1
