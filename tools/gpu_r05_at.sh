#!/bin/bash
# r05 call AT: the fused top at a four-wave register budget (variants/top4: 128 VGPRs, 132 B scratch)
# against the default (178 VGPRs); chunk parity under the variant, then ecrecover+chunk+notary twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05at; mkdir -p $O
T="timeout -k 10"
GSV_LIB_PATH=variants/top4/libgsv.so $T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_configs.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base top4; do
    if [ $v = base ]; then unset GSV_LIB_PATH; else export GSV_LIB_PATH=variants/$v/libgsv.so; fi
    $T 300 python bench.py --legs ecrecover,chunk_root,notary --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); print('$v rep $rep: chunk', d['collation_GBps'], 'GB/s', d['chunk_root']['ms_per_step'], 'ms | notary', d['notary']['shards_per_s'])"
  done
done
