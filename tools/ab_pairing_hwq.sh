#!/bin/bash
# The N = 8 per-rank pairing batch (8,192 checks) with 4-8 batches in flight, against the number of
# hardware queues HIP gives the process (GPU_MAX_HW_QUEUES: 4 by default; streams beyond it share
# queues, so deeper pipelines stop adding concurrency).  GPU box, repo root.
set -o pipefail
for q in 4 8 16; do
  for lay in "auto" "4 0 0" "2 1 0"; do
    set -- $lay
    if [ "$1" = auto ]; then E=""; else E="GSV_BN_PAIRS_PER_LANE=$1 GSV_BN_FINAL3=$2 GSV_BN_MILLER2=$3"; fi
    echo "queues $q layout k/final3/miller2 = $lay"
    env GPU_MAX_HW_QUEUES=$q $E SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE=3,4,8 timeout -k 10 300 python tools/pairing_sweep.py 8192 > gpurun_out/hwq_${q}_${1}${2}${3}.txt 2>&1 || { tail gpurun_out/hwq_${q}_${1}${2}${3}.txt; exit 1; }
    grep checks gpurun_out/hwq_${q}_${1}${2}${3}.txt
  done
done
