#!/bin/bash
# Profiles the bench on the GPU box (run through gpurun from the repo root):
#   all            rocprofv3 --kernel-trace --stats over the default bench      -> kernel_stats.csv
#   per leg G in {ecrecover, chunk_root, keccak, pairing, notary}: the leg ALONE, single stream
#   (--pipeline 1 --pairing-pipeline 1 --notary-pipeline 1 --ecrecover-pipeline 1, so no dispatch overlaps another batch's and the trace
#   average is the kernel's own duration), each counter set in its own pass:
#        --kernel-trace                                               -> durations
#        FETCH_SIZE / WRITE_SIZE                                      -> HBM bytes per dispatch
#        SQ_* VALU / wait counters + GRBM_GUI_ACTIVE                  -> issue rate, clock, stalls
#        SQ_INSTS_VALU_INT32 / _INT64                                 -> integer VALU instructions
# Output under gpurun_out/prof/<tag>/; summarised by tools/pmc_summary.py into pmc_<G>.json.
#   tools/profile_round.sh <tag> [groups...]   (default: all ecrecover chunk_root keccak pairing notary)
set -u
TAG=${1:-r03}
shift || true
GROUPS_=${*:-all ecrecover chunk_root keccak pairing notary}
OUT=gpurun_out/prof/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for G in $GROUPS_; do
    if [ $G = all ]; then
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/all/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
        find $OUT/all/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
        continue
    fi
    B="--legs $G --steps 3 --warmup 1 --no-cpu-baseline --pipeline 1 --pairing-pipeline 1 --notary-pipeline 1 --ecrecover-pipeline 1"
    # the notary step forks its chunk roots beside its transactions: no side streams in the leg-only
    # passes, so every traced dispatch runs alone (tools/pmc_summary.py drops any that still overlap)
    if [ $G = notary ]; then export GSV_MAX_SIDE_STREAMS=0; else unset GSV_MAX_SIDE_STREAMS; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f rocpd csv -d $OUT/$G/trace -o run -- python3 bench.py $B > $OUT/$G.trace.log 2>&1 || { echo "trace pass $G failed"; exit 1; }
    find $OUT/$G/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$G.csv \;
    # per-dispatch start / end of the library's kernels (small): tools/trace_agreement.py compares the
    # bench's instrumented launches with the same launches here (the first launches of a process read slow)
    python3 - $OUT/$G/trace $OUT/dispatch_$G.csv <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
rows = [r for r in csv.DictReader(open(f[0]))] if f else []
with open(sys.argv[2], "w") as o:
    o.write("kernel,start_ns,end_ns\n")
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        n = r["Kernel_Name"].split("(")[0]
        if "gsv::" in n:
            o.write(f"{n.replace(',', ';')},{r['Start_Timestamp']},{r['End_Timestamp']}\n")
PY
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/$G/fetch -o run -- python3 bench.py $B > $OUT/$G.fetch.log 2>&1 || { echo "fetch pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/$G/write -o run -- python3 bench.py $B > $OUT/$G.write.log 2>&1 || { echo "write pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/$G/sq -o run -- python3 bench.py $B > $OUT/$G.sq.log 2>&1 || { echo "sq pass $G failed"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE -d $OUT/$G/int -o run -- python3 bench.py $B > $OUT/$G.int.log 2>&1 || { echo "int pass $G failed"; exit 1; }
    python3 tools/pmc_summary.py $OUT/$G > $OUT/pmc_$G.json || { echo "summary $G failed"; exit 1; }
    echo "pass group $G done"
done
