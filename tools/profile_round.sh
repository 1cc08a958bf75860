#!/bin/bash
# Profiles the bench on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats on the full bench           -> per-kernel durations
#   2. per leg group G in {all, chunk_root, keccak}, each counter set in its own pass:
#        FETCH_SIZE / WRITE_SIZE                                      -> HBM bytes per dispatch
#        SQ_* VALU counters + GRBM_GUI_ACTIVE                         -> VALU issue rate
#        SQ_INSTS_VALU_INT32 / _INT64                                 -> integer VALU instructions
#      (chunk_root / keccak alone: their kernels are not averaged with the notary / POC dispatches
#       of the same kernels)
# Output under gpurun_out/prof/<tag>/; summarised by tools/pmc_summary.py into pmc_<G>.json.
set -u
TAG=${1:-r02}
BASE=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/all/trace -o run -- python3 bench.py $BASE > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
find $OUT/all/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
for G in all chunk_root keccak; do
    if [ $G = all ]; then LEGS=""; else LEGS="--legs $G"; fi
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/$G/fetch -o run -- python3 bench.py $BASE $LEGS > $OUT/$G.fetch.log 2>&1 || { echo "fetch pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/$G/write -o run -- python3 bench.py $BASE $LEGS > $OUT/$G.write.log 2>&1 || { echo "write pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/$G/sq -o run -- python3 bench.py $BASE $LEGS > $OUT/$G.sq.log 2>&1 || { echo "sq pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE -d $OUT/$G/int -o run -- python3 bench.py $BASE $LEGS > $OUT/$G.int.log 2>&1 || { echo "int pass $G failed"; exit 1; }
    if [ $G != all ]; then
        timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/$G/trace -o run -- python3 bench.py $BASE $LEGS > $OUT/$G.trace.log 2>&1 || { echo "trace pass $G failed"; exit 1; }
    fi
    python3 tools/pmc_summary.py $OUT/$G > $OUT/pmc_$G.json || { echo "summary $G failed"; exit 1; }
    echo "pass group $G done"
done
