#!/bin/bash
# A/B of the notary step's chunk roots forked onto a side stream (GSV_NOTARY_FORK): notary / partition /
# configs[3] GPU tests, then the notary leg alternating in-tree (fork) and variants/nofork.  GPU box.
set -o pipefail
O=gpurun_out/abfork
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_notary.py tests/test_gpu_partition.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_ARGS="--steps 12" timeout -k 10 600 python tools/ab_variants.py notary main nofork main nofork | tee $O/summary.txt || exit 1
