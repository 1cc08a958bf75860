#!/bin/bash
# r05 call J: which pipelined 8,192-check runs read slow, by stream identity (torch pool streams chosen
# explicitly), and the bench's pairing leg at the N = 8 per-rank batch with more timed steps
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05j; mkdir -p $O
T="timeout -k 10"
SWEEP_STREAM_SETS="0,1,2;0,1,2;3,4,5;0,1,2;1,2,3;2,3,4;4,5,6;0,4,8;0,1,2,3;4,5,6,7;0,1,2" $T 300 python -u tools/pairing_sweep.py 8192 > $O/stream_sets.txt 2>&1 && cat $O/stream_sets.txt
