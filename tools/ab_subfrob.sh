#!/bin/bash
# A/B of the G2 membership test taken from the line chain (BN_SUB_FROB, main) against the separate
# 63-bit psi check role (variants/nofrob): GPU tests (points in / outside G2, bad inputs, configs[4]
# verdicts, graph capture), the bench's pairing leg alternating, then the main library's sweep with the
# one-wave lines kernel (GSV_BN_CONC) forced off / on; last the chunk-root bottom-message A/B
# (variants/pz0).  GPU box, repo root.
set -o pipefail
O=gpurun_out/absub
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_bn256.py tests/test_gpu_configs.py tests/test_gpu_boundary.py tests/test_gpu_chunk_root.py -x -q --timeout 160 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
AB_ARGS="--steps 12" timeout -k 10 600 python tools/ab_variants.py pairing main nofrob main nofrob | tee $O/pairing.txt || exit 1
for c in 0 1; do
  GSV_BN_CONC=$c SWEEP_PIPELINE=1,2 timeout -k 10 400 python tools/pairing_sweep.py 8192 16384 65536 > $O/sweep_conc$c.txt 2>&1 || { echo "sweep $c failed"; tail -20 $O/sweep_conc$c.txt; exit 1; }
  echo "GSV_BN_CONC=$c"; cat $O/sweep_conc$c.txt
done
AB_ARGS="--pipeline 1 --steps 20" timeout -k 10 300 python tools/ab_variants.py chunk_root main pz0 main pz0 | tee $O/chunk_single_stream.txt || exit 1
