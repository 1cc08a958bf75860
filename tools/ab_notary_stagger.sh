#!/bin/bash
# The notary pipeline's step mark (GSV_NOTARY_STAGGER, gsv_api.hip notary_run): 1 = the chunk root's
# (after its bottom level, r03-r05), 0 = none, 2 = after the blob index; 13 / 25 / 100 shards (N = 8 / 4 /
# 1 rank shares of configs[3]) at depths 2-4, 12 and 40 steps per measurement, interleaved twice.  GPU box.
set -u
OUT=gpurun_out/ab_ns; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for st in 1 0 2; do
    for steps in 12 40; do
      GSV_NOTARY_STAGGER=$st NOTARY_DEPTHS=${DEPTHS:-2,3,4} NOTARY_STEPS=$steps timeout -k 10 200 \
        python3 tools/notary_sweep.py ${SHARDS:-13 25 100} > $OUT/s${st}_n${steps}_r$rep.txt 2>&1 || { echo "sweep failed"; tail $OUT/s${st}_n${steps}_r$rep.txt; exit 1; }
      echo "stagger $st steps $steps rep $rep"; grep shards $OUT/s${st}_n${steps}_r$rep.txt
    done
  done
done
