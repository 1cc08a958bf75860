#!/bin/bash
# r05 call F: the N = 8 rank batch (8,192 checks) pipelined three deep, repeated in ONE process: is the
# slow first depth-3 run (~6 ms per batch against ~3.8 later) a property of the first shape / streams
# of a process?  Also the bench's own pairing leg at 8,192 checks per rank (--pairing-checks).
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05f; mkdir -p $O
T="timeout -k 10"
SWEEP_PIPELINE="3,3,3,4,3,2,3" $T 300 python -u tools/pairing_sweep.py 8192 > $O/pipe_rep.txt 2>&1 || { echo pipe failed; tail $O/pipe_rep.txt; exit 1; }
grep checks $O/pipe_rep.txt
