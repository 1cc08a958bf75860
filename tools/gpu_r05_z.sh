#!/bin/bash
# r05 call Z: theta applied as one three-input XOR per word (GSV_KECCAK_THETA3, in-tree default) vs
# D first (variants/theta0): Keccak / chunk-root / notary / ecrecover parity tests, then A/B twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05z; mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_keccak.py tests/test_gpu_chunk_root.py tests/test_gpu_configs.py tests/test_gpu_collation.py tests/test_gpu_notary.py tests/test_gpu_secp256k1.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in theta3 theta0; do
    if [ $v = theta0 ]; then export GSV_LIB_PATH=variants/theta0/libgsv.so; else unset GSV_LIB_PATH; fi
    $T 300 python bench.py --legs ecrecover,chunk_root,notary,keccak --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); r=d['chunk_root']['roofline']; k=d['collation_extras']['keccak256']['roofline']; print('$v rep $rep: ecrecover', d['value'], '| chunk', d['collation_GBps'], 'GB/s bottom', r['kernel_avg_ms'], 'ms | keccak', k['kernel_avg_ms'], 'ms | notary', d['notary']['shards_per_s'])"
  done
done
