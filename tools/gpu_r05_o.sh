#!/bin/bash
# r05 call O: side streams on the context's own-queue pool - GPU tests, then on one box: the bench's
# pipelined legs with dedicated-queue streams vs torch pool streams (GSV_BENCH_TORCH_STREAMS=1), twice
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05o; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mode in own torch; do
    if [ $mode = torch ]; then export GSV_BENCH_TORCH_STREAMS=1; else unset GSV_BENCH_TORCH_STREAMS; fi
    $T 300 python bench.py --legs chunk_root,notary,pairing --no-cpu-baseline > $O/legs_${mode}_$rep.json 2> $O/legs_${mode}_$rep.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/legs_${mode}_$rep.json')); print('$mode rep $rep: chunk', d['collation_GBps'], 'GB/s | notary', d['notary']['shards_per_s'], '| pairing', d['bn256_pairing']['checks_per_s'], d['bn256_pairing']['ms_per_step'], 'ms')"
  done
done
