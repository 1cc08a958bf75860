#!/bin/bash
# Round-end evidence on the GPU box (repo root): op counts (instrumented build in variants/opcount), all
# GPU tests, smoke, the default bench, then tools/profile_round.sh (kernel trace + PMC passes).
set -o pipefail
mkdir -p gpurun_out/r02h
timeout -k 10 300 python -u tools/count_ops.py > gpurun_out/r02h/opcount.json 2> gpurun_out/r02h/opcount.err || { echo "opcount failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02h/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02h/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/r02h/bench.log 2>&1 || { echo "bench failed"; exit 1; }
bash tools/profile_round.sh r02h || { echo "profile failed"; exit 1; }
# keep the summaries (kernel_stats.csv, pmc_<group>.json, logs); the raw rocprofv3 output exceeds
# what gpurun copies back
find gpurun_out/prof/r02h -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
du -sh gpurun_out
echo all done
