#!/bin/bash
# The r05 exit-time SIGSEGV record (gpurun_out/r05l/sets_traced.txt): the pairing sweep over eight
# dedicated-queue streams under rocprofv3 --kernel-trace.  Since r06 the streams are the context's
# (gsv_stream_create) and every context closes at interpreter exit; the run must end with rc 0.  GPU box.
set -o pipefail
O=gpurun_out/exit_trace; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SWEEP_CUMASK=8 SWEEP_STREAM_SETS="0,1,2;1,2,3;0,4,7;0,1,2,3" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d $O/trace -o run -- python3 -u tools/pairing_sweep.py 8192 > $O/sets_traced.txt 2>&1
rc=$?
echo "rc $rc"; grep "streams " $O/sets_traced.txt; tail -3 $O/sets_traced.txt
exit $rc
