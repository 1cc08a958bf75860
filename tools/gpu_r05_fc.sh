#!/bin/bash
# r05 final evidence refresh after the bottom level's LDS stride change: the chunk_root leg-only passes,
# then GPU tests, smoke and the default bench -> gpurun_out/r05/bench.log (PMC summaries of the other
# legs are the committed ones in profiles/r05, unchanged kernels)
set -o pipefail
R=r05
O=gpurun_out/$R
mkdir -p $O
bash tools/profile_round.sh $R chunk_root || { echo "profile failed"; exit 1; }
cp gpurun_out/prof/$R/pmc_chunk_root.json gpurun_out/prof/$R/kernel_stats_chunk_root.csv profiles/$R/
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
echo final c done
