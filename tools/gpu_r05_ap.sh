#!/bin/bash
# r05 call AP: per-dispatch k_ecrecover durations in the leg-only trace pass (which launches read slow)
set -o pipefail
O=gpurun_out/r05ap; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/t -o run -- python3 bench.py --legs ecrecover --steps 3 --warmup 1 --no-cpu-baseline --ecrecover-pipeline 1 > $O/log.txt 2>&1 || { tail $O/log.txt; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05ap/t/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("gsv::k_ecrecover(")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
print(" ".join(f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:.3f}" for r in rows))
PY
grep '^{' $O/log.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench kernel_avg_ms', d['roofline']['kernel_avg_ms'])"
