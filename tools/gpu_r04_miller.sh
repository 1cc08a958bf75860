#!/bin/bash
# the same input bytes through the r04 and r03 libraries: inputs made by the r03 generator (old_in) and
# by the r04 generator (new_in, with the infinity / outside-G2 classes)
set -o pipefail
export PYTHONUNBUFFERED=1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_INPUT=/tmp/old_in.npz SWEEP_CASES="0,," timeout -k 10 200 python tools/pairing_sweep.py 65536 > /dev/null 2>&1 || exit 1
SWEEP_INPUT=/tmp/new_in.npz SWEEP_CASES="0,," timeout -k 10 200 python tools/pairing_sweep.py 65536 > /dev/null 2>&1 || exit 1
for rep in 1 2; do
for lib in new base_r03; do
  if [ $lib = new ]; then L=""; else L="GSV_LIB_PATH=variants/$lib/libgsv.so"; fi
  for inp in old_in new_in; do
    echo "== $lib $inp"; env $L SWEEP_INPUT=/tmp/$inp.npz SWEEP_CASES="0,," timeout -k 10 200 python tools/pairing_sweep.py 65536 8192 2>&1 | grep -E "checks|Error" || exit 1
  done
done
done
rm -f /tmp/old_in.npz /tmp/new_in.npz
