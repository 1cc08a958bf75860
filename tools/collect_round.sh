#!/bin/bash
# Local (CPU) step after tools/round_profile_a.sh and _b.sh ran on the GPU box: copy the round's
# evidence from gpurun_out/ into profiles/<round>/ (op counts, GPU test log, smoke, default bench, the
# leg-only kernel traces and PMC summaries, the bench line printed under each trace) and compute the
# HIP-event vs rocprofv3 agreement.   tools/collect_round.sh r05
set -euo pipefail
R=$1
P=profiles/$R
mkdir -p $P/trace_logs
for f in opcount.json gpu_tests.log smoke.log bench.log; do
  [ -f gpurun_out/$R/$f ] && cp gpurun_out/$R/$f $P/
done
cp gpurun_out/prof/$R/pmc_*.json gpurun_out/prof/$R/kernel_stats*.csv $P/
ls gpurun_out/prof/$R/dispatch_*.csv >/dev/null 2>&1 && cp gpurun_out/prof/$R/dispatch_*.csv $P/trace_logs/
for G in ecrecover chunk_root keccak pairing notary; do
  L=gpurun_out/prof/$R/$G.trace.log
  [ -f $L ] && grep '^{' $L | tail -1 > $P/trace_logs/bench_under_trace_$G.json
done
python3 tools/trace_agreement.py $P > $P/trace_agreement.json
echo collected into $P
