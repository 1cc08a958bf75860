#!/bin/bash
# Ad-hoc PMC passes over one bench leg (run through gpurun from the repo root):
#   tools/pmc_probe.sh <leg> <tag> "<counters pass 1>" ["<counters pass 2>" ...]
# Each pass is its own rocprofv3 run; per-kernel sums/means land in gpurun_out/probe/<tag>/summary.txt.
set -u
LEG=$1; TAG=$2; shift 2
OUT=gpurun_out/probe/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
i=0
for C in "$@"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $C -f csv -d $OUT/p$i -o run -- python3 bench.py --legs $LEG --steps 1 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - $OUT > $OUT/summary.txt <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} dispatches={len(v):4d} mean={sum(v)/len(v):.4g}")
PY
cat $OUT/summary.txt
