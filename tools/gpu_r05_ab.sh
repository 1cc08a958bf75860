#!/bin/bash
# r05 call AB: the bottom level's LDS message stride 88 / 104 bytes (variants bb88, bb104: 16 banks per
# wave) against 96 (4 banks); chunk parity under each first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05ab; mkdir -p $O
T="timeout -k 10"
for v in bb88 bb104; do
  GSV_LIB_PATH=variants/$v/libgsv.so $T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_configs.py > $O/tests_$v.log 2>&1; rc=$?; tail -1 $O/tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in base bb88 bb104; do
    if [ $v = base ]; then unset GSV_LIB_PATH; else export GSV_LIB_PATH=variants/$v/libgsv.so; fi
    $T 300 python bench.py --legs ecrecover,chunk_root --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); r=d['chunk_root']['roofline']; print('$v rep $rep: chunk', d['collation_GBps'], 'GB/s bottom', r['kernel_avg_ms'], 'ms')"
  done
done
