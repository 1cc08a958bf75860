"""Timeline of the last dispatches in a rocprofv3 kernel-trace CSV (pipelined `_dev` calls).

    python tools/trace_timeline.py <run_kernel_trace.csv> [--match SUBSTR ...] [--last K] [--anchor NAME]
        [--steps S]

Prints, for the last S steps (a step starts at each dispatch whose name contains --anchor), every
dispatch relative to the first one shown: start, end, duration, queue id, waves, registers.  Then the
span per step, how often 0 / 1 / 2 / ... of the matched kernels run at once, the per-kernel average
duration inside the pipeline, and the wave-milliseconds the matched kernels hold against the 1,024
SIMDs x the span (a kernel's waves x its duration, so a lower bound on occupancy, not a measurement).
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", nargs="*", default=[])
    ap.add_argument("--anchor", default="k_blob_index")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--quiet", action="store_true", help="no per-dispatch lines")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        n = r["Kernel_Name"].split("(")[0]
        if a.match and not any(m in n for m in a.match):
            continue
        waves = (int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1) + 63) // 64
        regs = int(r.get("VGPR_Count", 0) or 0) + int(r.get("Accum_VGPR_Count", 0) or 0)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r.get("Queue_Id", "?"), waves, regs))
    rows.sort()
    anchors = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    if len(anchors) < a.steps + 1:
        print(f"only {len(anchors)} anchors ({a.anchor})")
        return
    first = anchors[-a.steps - 1]
    sel = rows[first:]
    # the span of the last S steps: anchor to anchor, closing at the last anchor + one step
    t0 = rows[anchors[-a.steps - 1]][0]
    t1 = rows[anchors[-1]][0]
    span = t1 - t0
    if not a.quiet:
        for s, e, n, q, w, regs in sel:
            print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f}  q{q:>3s} w{w:7d} r{regs:4d}  {n[-48:]}")
    print(f"span {span / 1e6:.3f} ms over {a.steps} steps = {span / a.steps / 1e6:.3f} ms per step")
    inside = [r for r in sel if r[0] < t1]
    ev = sorted([(max(s, t0), 1) for s, e, *_ in inside] + [(min(e, t1), -1) for s, e, *_ in inside])
    cur, last, hist = 0, t0, collections.Counter()
    for t, d in ev:
        hist[cur] += t - last
        cur += d
        last = t
    for k in sorted(hist):
        print(f"  {k} kernels running: {hist[k] / span:.3f}")
    avg = collections.defaultdict(list)
    wt = 0.0
    for s, e, n, q, w, regs in inside:
        d = (min(e, t1) - max(s, t0)) / 1e6
        avg[(n, w, regs)].append((e - s) / 1e6)
        wt += w * d
    for (n, w, regs), v in sorted(avg.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[-44:]:44s} n={len(v):3d} waves {w:6d} regs {regs:4d} avg {sum(v) / len(v):.4f} ms")
    print(f"wave-ms held {wt:.1f} / (span x 1024 SIMDs) {span / 1e6 * 1024:.1f} = {wt / (span / 1e6 * 1024):.3f}")
    print("queues", dict(collections.Counter(r[3] for r in inside)))


if __name__ == "__main__":
    main()
