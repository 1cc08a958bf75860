#!/bin/bash
# Notary partition steps kept in flight on two streams (bench.py --notary-pipeline): partition / notary /
# configs[3] GPU tests, then the per-rank step time against the shards a rank holds
# (tools/notary_sweep.py), then the bench's notary leg at depth 1 and 2, alternating.  GPU box.
set -o pipefail
O=gpurun_out/abnpipe
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_notary.py tests/test_gpu_configs.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/notary_sweep.py 13 25 50 100 > $O/sweep.txt 2>&1 || { tail $O/sweep.txt; exit 1; }
grep shards $O/sweep.txt
for d in 1 2 1 2; do
  AB_ARGS="--steps 12 --notary-pipeline $d" timeout -k 10 300 python tools/ab_variants.py notary main | sed "s/^/depth $d: /" || exit 1
done
