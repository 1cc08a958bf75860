#!/bin/bash
# A/B of the fused trie top (k_chunk_top) on the chunk-root leg: parity tests per variant, then the
# leg on one stream (single-batch latency) and with the default two-stream pipeline; finally the
# per-height s_memtime trace (GSV_TOP_TRACE builds) of one 100 x 1 MiB batch.  GPU box, repo root.
set -o pipefail
O=gpurun_out/abtop
mkdir -p $O
for v in main "$@"; do
  if [ $v = main ]; then L=""; else L="variants/$v/libgsv.so"; fi
  GSV_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_chunk_root.py tests/test_gpu_configs.py -k "chunk or configs2" -x -q --timeout 120 --timeout-method thread > $O/test_$v.log 2>&1 || { echo "$v tests failed"; exit 1; }
done
AB_ARGS="--pipeline 1 --steps 20" timeout -k 10 300 python tools/ab_variants.py chunk_root main "$@" main "$@" | tee $O/single_stream.txt || exit 1
AB_ARGS="--steps 20" timeout -k 10 300 python tools/ab_variants.py chunk_root main "$@" | tee $O/pipelined.txt || exit 1
for v in toptr top4tr; do
  [ -d variants/$v ] || continue
  GSV_LIB_PATH=variants/$v/libgsv.so timeout -k 10 120 python -c "
import sys, numpy as np, torch
sys.path.insert(0, 'geth-sharding_amd')
import gsv
ctx = gsv.default_context()
b = torch.from_numpy(np.random.default_rng(1).integers(0, 256, 100 << 20, dtype=np.uint8)).cuda()
off = np.arange(101, dtype=np.uint64) << 20
r = torch.empty((100, 32), dtype=torch.uint8, device='cuda')
for _ in range(3):
    ctx.chunk_root_batch_dev(b, off, r)
torch.cuda.synchronize()
" > $O/trace_$v.txt 2>&1 || exit 1
done
echo done
