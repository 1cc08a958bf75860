#!/bin/bash
# Round-end evidence, part 1 (GPU box, repo root): op counts (instrumented build in variants/opcount),
# all GPU tests, smoke, the default bench's kernel trace and the ecrecover / chunk_root / keccak
# leg-only PMC passes (tools/profile_round.sh).  Part 2: tools/round_profile_b.sh.
set -o pipefail
R=${1:-r04}
O=gpurun_out/$R
mkdir -p $O
if [ -f variants/opcount/libgsv.so ]; then
  timeout -k 10 300 python -u tools/count_ops.py > $O/opcount.json 2> $O/opcount.err || { echo "opcount failed"; exit 1; }
else
  echo "no variants/opcount build: op counts not re-measured (profiles/<round>/opcount.json kept)"
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/profile_round.sh $R all ecrecover chunk_root keccak || { echo "profile failed"; exit 1; }
find gpurun_out/prof/$R -mindepth 1 -maxdepth 1 -type d -exec rm -rf {} +
echo part a done
