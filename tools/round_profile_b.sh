#!/bin/bash
# Round-end evidence, part 2 (GPU box, repo root): the pairing / notary leg-only PMC passes, then the
# default bench AFTER every PMC summary is in profiles/<round>/ of this tree (part 1's summaries were
# copied there before this call), so bench.log reads the passes committed beside it.
set -o pipefail
R=${1:-r04}
O=gpurun_out/$R
mkdir -p $O profiles/$R
bash tools/profile_round.sh $R pairing notary || { echo "profile failed"; exit 1; }
cp gpurun_out/prof/$R/pmc_*.json gpurun_out/prof/$R/kernel_stats*.csv profiles/$R/
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; exit 1; }
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
echo part b done
