#!/bin/bash
# Round-end evidence on the GPU box (repo root): op counts (instrumented build in variants/opcount), all
# GPU tests, smoke, tools/profile_round.sh (kernel traces + leg-only PMC passes), then the default bench
# AFTER the PMC summaries are in profiles/<round>/ of this tree, so bench.log reads the passes beside it.
set -o pipefail
R=${1:-r03}
O=gpurun_out/$R
mkdir -p $O profiles/$R
timeout -k 10 300 python -u tools/count_ops.py > $O/opcount.json 2> $O/opcount.err || { echo "opcount failed"; exit 1; }
cp $O/opcount.json profiles/$R/opcount.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/profile_round.sh $R || { echo "profile failed"; exit 1; }
cp gpurun_out/prof/$R/pmc_*.json gpurun_out/prof/$R/kernel_stats*.csv profiles/$R/
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
# keep the summaries (kernel_stats*.csv, pmc_<group>.json, logs); the raw rocprofv3 output exceeds
# what gpurun copies back
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
du -sh gpurun_out
echo all done
