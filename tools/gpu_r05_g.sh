#!/bin/bash
# r05 call G: pairing tests with the batch-size rule for the two-wave lines kernel; the first-run
# artifact of the pipelined N = 8 batch with the GPU pre-heated for 1.5 s
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05g; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest tests/test_gpu_bn256.py "tests/test_gpu_configs.py::test_configs4_full_batch_verdicts" \
   -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SWEEP_PREHEAT=1 SWEEP_PIPELINE="3,3,4,3" $T 300 python -u tools/pairing_sweep.py 8192 > $O/pipe_preheat.txt 2>&1 || { echo pipe failed; tail $O/pipe_preheat.txt; exit 1; }
grep checks $O/pipe_preheat.txt
SWEEP_PIPELINE="2,2,3" $T 300 python -u tools/pairing_sweep.py 65536 > $O/pipe_65536.txt 2>&1 || { echo pipe failed; tail $O/pipe_65536.txt; exit 1; }
grep checks $O/pipe_65536.txt
