#!/bin/bash
# r05 call X: chunk-root pipeline with the tail mark after the bottom level (GSV_CHUNK_TAIL_BOTTOM=1) vs
# before the fused top; chunk tests under the switch first
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05x; mkdir -p $O
T="timeout -k 10"
GSV_CHUNK_TAIL_BOTTOM=1 $T 300 python -u -m pytest -x -q --timeout 160 --timeout-method thread -m gpu tests/test_gpu_chunk_root.py tests/test_gpu_boundary.py > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for tb in 0 1; do
    for d in 2 3; do
      GSV_CHUNK_TAIL_BOTTOM=$tb $T 300 python bench.py --legs chunk_root,notary --pipeline $d --no-cpu-baseline > $O/cr_t${tb}_d${d}_$rep.json 2> $O/cr_t${tb}_d${d}_$rep.err || exit 1
      python3 -c "
import json; d=json.load(open('$O/cr_t${tb}_d${d}_$rep.json')); print('tail_bottom $tb depth $d rep $rep: chunk', d['collation_GBps'], 'GB/s', d['chunk_root']['ms_per_step'], 'ms | notary', d['notary']['shards_per_s'])"
    done
  done
done
