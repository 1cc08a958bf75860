#!/bin/bash
# r05 call L: pipelined 8,192-check runs over CU-masked streams (each its own HSA queue?) - timings and
# the kernel trace's queue ids
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05l; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SWEEP_CUMASK=8 SWEEP_STREAM_SETS="0,1,2;1,2,3;4,5,6;0,4,7;0,1,2,3;4,5,6,7" timeout -k 10 300 python3 -u tools/pairing_sweep.py 8192 > $O/sets.txt 2>&1 && grep streams $O/sets.txt && \
SWEEP_CUMASK=8 SWEEP_STREAM_SETS="0,1,2;1,2,3;0,4,7;0,1,2,3" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 -u tools/pairing_sweep.py 8192 > $O/sets_traced.txt 2>&1 && grep "streams " $O/sets_traced.txt
