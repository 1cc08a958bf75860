#!/bin/bash
# Profiles the bench command on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats            -> per-kernel durations
#   2. rocprofv3 --pmc FETCH_SIZE   (own pass)     -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE   (own pass)     -> HBM write bytes per dispatch
#   4. rocprofv3 --pmc SQ_* VALU counters          -> VALU busy / instruction mix
# Output under gpurun_out/prof/<tag>/; summarised by tools/pmc_summary.py.
set -u
TAG=${1:-r01}
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || { echo "write pass failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
find $OUT -name "*.csv" | head -50
# the kernel-trace --stats CSV summary lands next to the db (run_kernel_stats.csv)
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
