#!/bin/bash
# Kernel trace of 8,192-check pairing batches at pipeline depth 4 (work-efficient layout k = 4, one-lane
# final): per-kernel durations and how many pairing kernels run at once over the timed region.  GPU box.
set -u
OUT=gpurun_out/trace_pp
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
GSV_BN_PAIRS_PER_LANE=4 GSV_BN_FINAL3=0 GSV_BN_MILLER2=0 SWEEP_KEEP_LAYOUT=1 SWEEP_PIPELINE=${DEPTH:-4} timeout -k 10 300 \
    rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 tools/pairing_sweep.py 8192 > $OUT/log.txt 2>&1 || { echo "trace failed"; tail $OUT/log.txt; exit 1; }
grep checks $OUT/log.txt
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/trace_pp/**/run_kernel_trace.csv", recursive=True)[0]
rows = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""), r.get("Stream_Id", ""))
        for r in csv.DictReader(open(f))]
rows = [r for r in rows if "bn::k_bn" in r[0] and "synth" not in r[0]]
rows.sort(key=lambda r: r[1])
tail = rows[-36:]  # the last 12 batches x 3 kernels
t0, t1 = min(r[1] for r in tail), max(r[2] for r in tail)
ev = sorted([(s, 1) for _, s, _, _, _ in tail] + [(e, -1) for _, _, e, _, _ in tail])
cur = 0; last = t0; hist = collections.Counter()
for t, d in ev:
    hist[cur] += t - last; cur += d; last = t
span = t1 - t0
print(f"span {span/1e6:.2f} ms for 12 batches = {span/12/1e6:.2f} ms per batch")
for k in sorted(hist): print(f"  {k} kernels running: {hist[k]/span:.3f}")
avg = collections.defaultdict(list)
for n, s, e, q, st in tail: avg[n].append((e - s) / 1e6)
for n, v in avg.items(): print(f"  {n[-24:]:24s} avg {sum(v)/len(v):.3f} ms")
print("queues:", sorted(set(r[3] for r in tail)), "streams:", sorted(set(r[4] for r in tail)))
for n, s, e, q, st in tail[:12]: print(f"  {n[-14:]:14s} q{q} s{st} {(s-t0)/1e6:8.3f} -> {(e-t0)/1e6:8.3f}")
PY
