#!/bin/bash
# r05 call AA: chunk-root level kernels at five waves per SIMD (variants/lw5, 96 VGPRs) and the Keccak
# round loop unrolled by two (variants/ku2) against the in-tree library; chunk parity under each first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05aa; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 160 --timeout-method thread -m gpu tests/test_gpu_boundary.py -k "capture" > $O/tests_capture.log 2>&1; echo "capture tests rc=$?"; grep -E "PASS|FAIL|Error|error" $O/tests_capture.log | head -12
for v in lw5 ku2; do
  GSV_LIB_PATH=variants/$v/libgsv.so $T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_keccak.py > $O/tests_$v.log 2>&1; rc=$?; tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in base lw5 ku2; do
    if [ $v = base ]; then unset GSV_LIB_PATH; else export GSV_LIB_PATH=variants/$v/libgsv.so; fi
    $T 300 python bench.py --legs chunk_root,keccak --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); r=d['chunk_root']['roofline']; k=d['collation_extras']['keccak256']['roofline']; print('$v rep $rep: chunk', d['collation_GBps'], 'GB/s bottom', r['kernel_avg_ms'], 'ms | keccak', k['kernel_avg_ms'], 'ms')"
  done
done
