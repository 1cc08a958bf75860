#!/bin/bash
# Kernel trace of the chunk-root leg alone at pipeline depth 1 and 2: per-kernel average duration, the
# step time, and how much of the step the GPU spent with no chunk kernel running (gaps) — where a
# two-stream step loses against the sum of its bulk kernels.  GPU box, repo root.
set -u
OUT=gpurun_out/trace_cp
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for d in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/d$d -o run -- python3 bench.py --legs chunk_root \
      --no-cpu-baseline --steps 20 --pipeline $d > $OUT/log_d$d.txt 2>&1 || { echo "trace failed"; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for d in (1, 2):
    f = glob.glob(f"gpurun_out/trace_cp/d{d}/**/run_kernel_trace.csv", recursive=True)[0]
    rows = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(f))]
    rows = [r for r in rows if "chunk" in r[0]]
    rows.sort(key=lambda r: r[1])
    # the timed region: the last 20 bottom launches and what overlaps them
    bots = [r for r in rows if r[0].endswith("k_chunk_level<true>")]
    t0, t1 = bots[-20][1], max(e for _, _, e in rows)
    sel = [r for r in rows if r[2] > t0]
    busy, last = 0, t0
    for _, s, e in sorted(sel, key=lambda r: r[1]):
        s = max(s, t0)
        if e <= last:
            continue
        busy += e - max(s, last)
        last = e
    span = t1 - t0
    avg = collections.defaultdict(list)
    for n, s, e in sel:
        avg[n].append((e - s) / 1e6)
    print(f"depth {d}: span per step {span / 20 / 1e6:.3f} ms, GPU busy {busy / span:.3f} of it")
    for n, v in sorted(avg.items()):
        print(f"   {n[-40:]:40s} n={len(v):4d} avg {sum(v) / len(v):.4f} ms")
PY
