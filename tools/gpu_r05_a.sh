#!/bin/bash
# r05 call A: new tests (stream contract, >4 GiB workspace, keccak staging) + the pairing / Miller
# sweep with the two-wave Miller kernel on and off + the Keccak kernel's scale sweep (staged, direct,
# r04 kernel)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05a; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream_contract.py \
   tests/test_gpu_keccak.py tests/test_gpu_bn256.py "tests/test_gpu_configs.py::test_configs4_full_batch_verdicts" \
   > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in 1 0; do
  GSV_BN_MILLER_W2=$w SWEEP_CASES="0,,;4,,;2,,;1,," $T 240 python -u tools/pairing_sweep.py 65536 8192 > $O/sweep_w$w.txt 2>&1 || { echo sweep $w failed; tail $O/sweep_w$w.txt; exit 1; }
  GSV_BN_MILLER_W2=$w SWEEP_PIPELINE="2,3" $T 240 python -u tools/pairing_sweep.py 65536 16384 8192 >> $O/sweep_w$w.txt 2>&1 || { echo pipe $w failed; tail $O/sweep_w$w.txt; exit 1; }
  grep checks $O/sweep_w$w.txt | sed "s/^/w2=$w /"
done
for v in base kec0 kold; do
  if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L $T 200 python -u tools/keccak_scale.py 400000 1600000 6400000 > $O/kscale_$v.txt 2>&1 || { echo kscale $v failed; tail $O/kscale_$v.txt; exit 1; }
  grep messages $O/kscale_$v.txt | sed "s/^/$v /"
done
