#!/bin/bash
# Kernel trace of the chunk-root leg only (gpurun from the repo root): per-dispatch durations.
set -u
OUT=gpurun_out/trace_chunk
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 bench.py --workload chunk_root --steps 3 --warmup 1 --no-cpu-baseline > $OUT/log.txt 2>&1 || { echo "trace failed"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/trace_chunk/**/run_kernel_trace.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "chunk" in r["Kernel_Name"] or "derive" in r["Kernel_Name"]:
        print(r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], r["VGPR_Count"], r["Scratch_Size"],
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, "us")
PY
