#!/bin/bash
# Kernel trace of the N = 8 per-rank notary step (configs[3]: 13 shards of 8,192 txs) pipelined
# DEPTHS deep on dedicated-queue streams (tools/notary_sweep.py), one profiled process per depth, and the
# timeline of the last steps (tools/trace_timeline.py).  GPU box, repo root.
set -u
OUT=gpurun_out/trace_np
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
SH=${SHARDS:-13}
for d in ${DEPTHS:-3 4}; do
  NOTARY_DEPTHS=$d NOTARY_NO_TIMING=1 NOTARY_STEPS=24 timeout -k 10 240 \
    rocprofv3 --kernel-trace -f csv -d $OUT/d$d -o run -- python3 tools/notary_sweep.py $SH > $OUT/log_d$d.txt 2>&1 \
    || { echo "trace d$d failed"; tail $OUT/log_d$d.txt; exit 1; }
  cat $OUT/log_d$d.txt | grep shards
  f=$(python3 -c "import glob; print(glob.glob('$OUT/d$d/**/run_kernel_trace.csv', recursive=True)[0])")
  python3 tools/trace_timeline.py $f --anchor k_blob_index --steps 8 > $OUT/timeline_d$d.txt
  tail -16 $OUT/timeline_d$d.txt
done
