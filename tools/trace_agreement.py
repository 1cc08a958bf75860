"""Does the bench's own kernel time (HIP events on the launching stream) agree with rocprofv3's kernel
trace of the SAME run?  For each leg traced alone by tools/profile_round.sh, compares the kernel
average the traced bench printed (profiles/<round>/trace_logs/bench_under_trace_<leg>.json) with the
trace's average for that kernel (profiles/<round>/kernel_stats_<leg>.csv).

    python tools/trace_agreement.py profiles/r03 > profiles/r03/trace_agreement.json
"""
import csv
import json
import os
import sys

LEGS = {  # leg: (kernel name prefix in the trace, how to read the bench's HIP-event average)
    "ecrecover": ("gsv::k_ecrecover", lambda d: d["roofline"]["kernel_avg_ms"]),
    "chunk_root": ("void gsv::k_chunk_level<true>", lambda d: d["chunk_root"]["bottom_kernel_avg_ms"]),
    "keccak": ("gsv::k_keccak256", lambda d: d["collation_extras"]["keccak256"]["roofline"]["kernel_avg_ms"]),
    "pairing:prepare": ("gsv::bn::k_bn_lines", lambda d: d["bn256_pairing"]["prepare_kernel_ms"]),
    "pairing:miller": ("gsv::bn::k_bn_miller", lambda d: d["bn256_pairing"]["miller_kernel_ms"]),
    "pairing:final": ("gsv::bn::k_bn_final", lambda d: d["bn256_pairing"]["final_exp_kernel_ms"]),
}


def main(root):
    out = {}
    for key, (kname, get) in LEGS.items():
        leg = key.split(":")[0]
        try:
            with open(os.path.join(root, "trace_logs", f"bench_under_trace_{leg}.json")) as f:
                bench_ms = get(json.loads(f.read()))
            with open(os.path.join(root, f"kernel_stats_{leg}.csv")) as f:
                allrows = list(csv.DictReader(f))
            # the pairing's lines kernel runs as k_bn_lines_w2 at large batches (r05): either name
            rows = [r for r in allrows if r["Name"].startswith(kname + "(")] or \
                [r for r in allrows if r["Name"].startswith(kname + "_w2(")]
        except (OSError, KeyError, ValueError):
            continue
        if not rows:
            continue
        prof_ms = float(rows[0]["AverageNs"]) / 1e6
        kname_full = rows[0]["Name"].split("(")[0]
        out[key] = {"kernel": kname_full, "bench_hip_event_ms": bench_ms, "rocprofv3_avg_ms": round(prof_ms, 4),
                    "calls": int(rows[0]["Calls"]), "ratio": round(bench_ms / prof_ms, 4)}
        # the same launches on both sides where the bench names its instrumented launch count (the last
        # launches of its leg): the trace's first launches of a process read slow (clock ramp-up)
        try:
            with open(os.path.join(root, "trace_logs", f"bench_under_trace_{leg}.json")) as f:
                n = json.loads(f.read())["roofline"].get("kernel_launches_timed") if leg == "ecrecover" else None
            with open(os.path.join(root, "trace_logs", f"dispatch_{leg}.csv")) as f:
                d = [r for r in csv.DictReader(f) if r["kernel"] == kname_full]
        except (OSError, KeyError, ValueError):
            n, d = None, []
        if n and len(d) >= n:
            last = sum(int(r["end_ns"]) - int(r["start_ns"]) for r in d[-n:]) / n / 1e6
            out[key].update({"rocprofv3_same_launches_ms": round(last, 4), "same_launches": n,
                             "ratio_same_launches": round(bench_ms / last, 4)})
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
