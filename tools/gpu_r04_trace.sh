#!/bin/bash
# kernel trace of the pairing sweep (65,536 then 8,192 checks) for this library and r03 on the same
# input bytes (made by the r03 generator): kernel durations independent of the library's own timers
set -o pipefail
export PYTHONUNBUFFERED=1
GSV_LIB_PATH=variants/base_r03/libgsv.so SWEEP_INPUT=/tmp/old_in.npz SWEEP_CASES="0,," timeout -k 10 200 python tools/pairing_sweep.py 65536 > /dev/null 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in new base_r03; do
  if [ $lib = new ]; then L=""; else L="$GRAFT_REPO_ROOT/variants/$lib/libgsv.so"; fi
  GSV_LIB_PATH=$L SWEEP_INPUT=/tmp/old_in.npz SWEEP_CASES="0,," timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/prof_$lib -o run -- python3 $GRAFT_REPO_ROOT/tools/pairing_sweep.py 65536 8192 > /tmp/prof_$lib.log 2>&1 || { tail /tmp/prof_$lib.log; exit 1; }
  echo "== $lib"; grep checks /tmp/prof_$lib.log
  f=$(find /tmp/prof_$lib -name "*kernel_stats.csv" | head -1); grep -E "bn_" "$f" | cut -d, -f1-8
  t=$(find /tmp/prof_$lib -name "*kernel_trace.csv" | head -1); cp "$t" $GRAFT_REPO_ROOT/gpurun_out/g7_trace_$lib.csv
done
