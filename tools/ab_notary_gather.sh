#!/bin/bash
# A/B of k_notary_tx's preimage / r / s reads (run through gpurun from the repo root):
#   base = in-tree: blob bytes gathered as dwords through the chunk map (BlobView::dword), loads issued
#          together, suffix from a zero-padded buffer
#   nold = the r06 library before it (one dependent byte load per preimage / r / s byte), variants/nold
# Notary GPU tests on the in-tree library; then per library, twice in alternation: one step at a time
# with no side streams (tx kernels alone, 100 and 128 shards) and the bench's notary leg (defaults).
set -o pipefail
O=gpurun_out/ng; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_notary.py tests/test_gpu_partition.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in base nold; do
    if [ $v = base ]; then L=""; else L="variants/$v/libgsv.so"; fi
    GSV_LIB_PATH=$L GSV_MAX_SIDE_STREAMS=0 NOTARY_DEPTHS=1 NOTARY_STEPS=12 timeout -k 10 300 python3 tools/notary_sweep.py 128 100 > $O/${v}_r$rep.txt 2>&1 || { echo "$v sweep failed"; tail $O/${v}_r$rep.txt; exit 1; }
    grep shards $O/${v}_r$rep.txt | sed "s/^/$v /"
    GSV_LIB_PATH=$L timeout -k 10 300 python3 bench.py --legs notary --no-cpu-baseline > $O/bench_${v}_r$rep.log 2>&1 || { echo "$v bench failed"; tail -5 $O/bench_${v}_r$rep.log; exit 1; }
    tail -1 $O/bench_${v}_r$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['notary']; print('$v leg', d['shards_per_s'], 'shards/s', d.get('ms_per_step'), 'ms/step')"
  done
done
