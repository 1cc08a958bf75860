#!/bin/bash
# Per-dispatch kernel durations of a bench run (gpurun from the repo root):
#   bash tools/trace_kernels.sh <name-filter-regex> [bench args...]
set -u
FILTER=$1; shift
OUT=gpurun_out/trace_k
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 bench.py "$@" > $OUT/log.txt 2>&1 || { echo "trace failed"; exit 1; }
python3 - "$FILTER" <<'PY'
import csv, glob, re, sys
f = glob.glob("gpurun_out/trace_k/**/run_kernel_trace.csv", recursive=True)[0]
pat = re.compile(sys.argv[1])
for r in csv.DictReader(open(f)):
    if pat.search(r["Kernel_Name"]):
        print(r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], r["Workgroup_Size_X"],
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, "us", int(r["Start_Timestamp"]) // 1000)
PY
