#!/bin/bash
# r05 final evidence, part 1: GPU tests, smoke, the default bench's kernel trace and the ecrecover /
# chunk_root / keccak leg-only PMC passes (tools/profile_round.sh); op counts unchanged (no
# multiply-add changed since profiles/r05/opcount.json).  Part 2: tools/round_profile_b.sh r05.
set -o pipefail
R=r05
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/profile_round.sh $R all ecrecover chunk_root keccak || { echo "profile failed"; exit 1; }
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
echo part a done
