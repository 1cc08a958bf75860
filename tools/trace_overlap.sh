#!/bin/bash
# Evidence of the two-stream pipeline: kernel trace of the chunk-root and pairing legs
# at pipeline depth 2, then for each latency-bound tail kernel (k_chunk_top, k_bn_miller, k_bn_final)
# the fraction of its duration during which another batch's bulk kernel (k_chunk_level<true>,
# k_bn_prepare) was running.  Run on the GPU box from the repo root.
set -u
OUT=gpurun_out/trace_ov
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT -o run -- python3 bench.py --legs chunk_root,pairing \
    --no-cpu-baseline --steps 12 --pipeline 2 --pairing-pipeline 2 > $OUT/log.txt 2>&1 || { echo "trace failed"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/trace_ov/**/run_kernel_trace.csv", recursive=True)[0]
rows = [(r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id", r.get("Queue_Id", "")))
        for r in csv.DictReader(open(f))]
def ov(tail, bulk):
    T = [r for r in rows if r[0].endswith(tail)]
    B = [r for r in rows if r[0].endswith(bulk)]
    tot = cov = 0
    for _, s, e, q in T:
        tot += e - s
        segs = sorted((max(s, bs), min(e, be)) for _, bs, be, bq in B if bs < e and be > s)
        last = s
        for a, b in segs:
            if b <= last:
                continue
            cov += b - max(a, last)
            last = b
    return len(T), tot / 1e3 / max(len(T), 1), cov / max(tot, 1)
for tail, bulk in (("k_chunk_top", "k_chunk_level<true>"), ("k_bn_miller", "k_bn_lines"), ("k_bn_final", "k_bn_lines")):
    n, avg, frac = ov(tail, bulk)
    print(f"{tail:14s} dispatches {n:3d}  avg {avg:9.1f} us  overlapped by {bulk}: {100 * frac:5.1f} % of its time")
PY
