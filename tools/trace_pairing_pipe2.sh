#!/bin/bash
# Kernel trace of the N = 8 per-rank pairing batch (8,192 checks) pipelined at DEPTH (default 4) on
# dedicated-queue streams with the AUTO layout: per-kernel durations inside the pipeline, how many
# pairing kernels run at once, and the wave-time the kernels hold against the 1,024 SIMDs (each pairing
# wave holds a SIMD alone: one-wave register budgets) over the last 12 batches.  GPU box.
set -u
OUT=gpurun_out/trace_pp2
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
SWEEP_PIPELINE=${DEPTH:-4} timeout -k 10 300 \
    rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 tools/pairing_sweep.py 8192 > $OUT/log.txt 2>&1 || { echo "trace failed"; tail $OUT/log.txt; exit 1; }
grep checks $OUT/log.txt
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/trace_pp2/**/run_kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0]
    if "bn::k_bn" not in n or "synth" in n:
        continue
    waves = int(r["Grid_Size_X"]) // 64
    rows.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), waves, r["Queue_Id"], int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"])))
rows.sort(key=lambda r: r[1])
tail = rows[-36:]
t0, t1 = min(r[1] for r in tail), max(r[2] for r in tail)
span = t1 - t0
ev = sorted([(s, 1) for _, s, _, _, _, _ in tail] + [(e, -1) for _, _, e, _, _, _ in tail])
cur = 0; last = t0; hist = collections.Counter()
for t, d in ev:
    hist[cur] += t - last; cur += d; last = t
print(f"span {span/1e6:.2f} ms for 12 batches = {span/12/1e6:.2f} ms per batch")
for k in sorted(hist): print(f"  {k} kernels running: {hist[k]/span:.3f}")
avg = collections.defaultdict(list)
wt = 0.0
for n, s, e, w, q, regs in tail:
    avg[(n, w, regs)].append((e - s) / 1e6)
for (n, w, regs), v in avg.items():
    d = sum(v) / len(v)
    print(f"  {n[-22:]:22s} waves {w:5d} regs {regs:4d} in-pipeline avg {d:.3f} ms  wave-ms per batch {w * d:.0f}")
    wt += w * d * len(v)
print(f"wave-ms held {wt:.0f} over span x 1024 SIMDs {span/1e6*1024:.0f}: {wt/(span/1e6*1024):.3f}")
qs = collections.Counter(q for _, _, _, _, q, _ in tail)
print("queues", dict(qs))
PY
