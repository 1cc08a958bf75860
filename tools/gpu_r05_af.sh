#!/bin/bash
# r05 call AF: HFULL child-hash prefetch (GSV_HF_PREFETCH, in-tree) vs none (variants/hfp0)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05af; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_configs.py tests/test_gpu_collation.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in hfp1 hfp0; do
    if [ $v = hfp1 ]; then unset GSV_LIB_PATH; else export GSV_LIB_PATH=variants/$v/libgsv.so; fi
    $T 300 python bench.py --legs ecrecover,chunk_root,notary,poc --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); c=d['chunk_root']; print('$v rep $rep: chunk', d['collation_GBps'], 'GB/s', c['ms_per_step'], 'ms, levels', c['level_kernels_ms_per_step'], 'ms | notary', d['notary']['shards_per_s'], '| poc', d['collation_extras']['proof_of_custody']['salted_GBps'])"
  done
done
