#!/bin/bash
# r05 call K: kernel trace (queue / stream ids, timelines) of pipelined 8,192-check runs over chosen
# pool streams: fast (0,1,2), slow (1,2,3), fast (4,5,6), slow (0,4,8)
set -o pipefail
export PYTHONUNBUFFERED=1
O=gpurun_out/r05k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SWEEP_STREAM_SETS="0,1,2;1,2,3;4,5,6;0,4,8" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 -u tools/pairing_sweep.py 8192 > $O/sets.txt 2>&1 && cat $O/sets.txt | grep -v "^\[" | tail -8 && find $O/trace -name "*.csv" | head
