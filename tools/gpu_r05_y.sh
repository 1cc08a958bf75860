#!/bin/bash
# r05 call Y: branch-free bottom-level leaf encoding (variants/botor, -DGSV_BOT_OR=1) - chunk-root
# parity tests under the variant, then configs[2] / notary A/B against the in-tree library, twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05y; mkdir -p $O
T="timeout -k 10"
GSV_LIB_PATH=variants/botor/libgsv.so $T 400 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_configs.py tests/test_gpu_collation.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base botor; do
    if [ $v = botor ]; then export GSV_LIB_PATH=variants/botor/libgsv.so; else unset GSV_LIB_PATH; fi
    $T 300 python bench.py --legs chunk_root,notary,poc --no-cpu-baseline > $O/${v}_$rep.json 2> $O/${v}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${v}_$rep.json')); r=d['chunk_root']['roofline']; print('$v rep $rep: chunk', d['collation_GBps'], 'GB/s', d['chunk_root']['ms_per_step'], 'ms, bottom', r['kernel_avg_ms'], 'ms | notary', d['notary']['shards_per_s'], '| poc', d['collation_extras']['proof_of_custody']['salted_GBps'])"
  done
done
