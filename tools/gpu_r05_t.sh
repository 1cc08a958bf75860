#!/bin/bash
# r05 call T (round-end refresh after the dedicated-queue streams): GPU tests, smoke, the default
# bench's kernel trace (all legs), then the default bench -> gpurun_out/r05/bench.log.  The leg-only
# PMC passes of parts A/B stay valid (kernels unchanged; they run one stream, depth 1).
set -o pipefail
export PYTHONUNBUFFERED=1
R=r05
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/profile_round.sh $R all || { echo "profile failed"; exit 1; }
cp gpurun_out/prof/$R/kernel_stats.csv profiles/$R/kernel_stats.csv
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('bench', d['value'], d['collation_GBps'], d['bn256_pairing']['checks_per_s'], d['notary']['shards_per_s'], d['roofline']['frac'])"
