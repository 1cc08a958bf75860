"""Summarise a tools/profile_round.sh run (rocprofv3 SQLite outputs) into one JSON per kernel.

    python tools/pmc_summary.py gpurun_out/prof/<tag>/<group> > profiles/<tag>/pmc_<group>.json

Per kernel: dispatches, average duration (kernel-trace pass), VGPR/scratch, HBM bytes per
dispatch from FETCH_SIZE and WRITE_SIZE (each from its own pass), SQ VALU counters and the
integer VALU instruction counts (SQ_INSTS_VALU_INT32 / _INT64).
gfx950 correction (MI355X_MICROARCH.md § HBM): FETCH_SIZE counts 64 B per 128-B request for
wide coalesced reads, so `fetch_bytes_x2` doubles it; which of the two applies depends on the
kernel's access width — both are reported, with the raw value.

Overlapped dispatches (r06): the counter passes serialise dispatches, but the
kernel-trace pass does not, so a dispatch that ran beside another in the trace pass (a forked chunk
root beside k_notary_tx) has a trace duration that is not its own, and any figure dividing its counters
by that duration is wrong (r05 pmc_notary.json: "clocks" of 0.054 and 5.7 GHz).  Dispatch i of a kernel
in the trace pass is paired with dispatch i of the same kernel in the SQ pass (the same program issues
them in the same order); a dispatch whose derived clock, GRBM_GUI_ACTIVE / 8 / its trace duration, lies
outside [CLK_LO, CLK_HI] GHz is dropped from every per-dispatch figure and counted in
"implausible_clock_dispatches" (an overlapped dispatch, or one too short for its counter window: a
~0.1 ms launch's GRBM_GUI_ACTIVE window includes the dispatch overhead).  A kernel with no plausible
dispatch keeps only its dispatch count and that count.
"""
import json
import os
import sqlite3
import sys
from collections import defaultdict


CLK_LO, CLK_HI = 1.0, 2.6  # GHz: MI355X runs 1.9-2.4 GHz under load (MI355X_MICROARCH.md, DVFS)


def short(name):
    return name.split("(")[0]


def counters(db, names):
    out = defaultdict(lambda: defaultdict(list))
    con = sqlite3.connect(db)
    for kname, cname, val, disp, vgpr, agpr, scratch in con.execute(
            "select kernel_name, counter_name, value, dispatch_id, vgpr_count, accum_vgpr_count, scratch_size "
            "from counters_collection"):
        if cname in names:
            out[short(kname)][cname].append((disp, val))
        out[short(kname)]["_res"] = [(0, (vgpr, agpr, scratch))]
    return out


def durations(db):
    con = sqlite3.connect(db)
    d = defaultdict(list)
    for kname, start, end in con.execute("select name, start, end from kernels order by start"):
        d[short(kname)].append(end - start)
    return d


def by_dispatch(vals):
    """per-dispatch sums (SQ counters arrive per shader engine), in dispatch order"""
    agg = defaultdict(float)
    for disp, v in vals:
        agg[disp] += v
    return [agg[d] for d in sorted(agg)]


def per_dispatch(vals, keep=None):
    """average over the kept dispatches (keep: indices in dispatch order; None = all)"""
    xs = by_dispatch(vals)
    if keep is not None:
        xs = [x for i, x in enumerate(xs) if i in keep]
    return sum(xs) / max(len(xs), 1)


def main(root):
    res = {}
    dur = durations(os.path.join(root, "trace", "run_results.db"))
    fetch = counters(os.path.join(root, "fetch", "run_results.db"), {"FETCH_SIZE"})
    write = counters(os.path.join(root, "write", "run_results.db"), {"WRITE_SIZE"})
    sq = counters(os.path.join(root, "sq", "run_results.db"),
                  {"SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
                   "GRBM_GUI_ACTIVE", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"})
    ipath = os.path.join(root, "int", "run_results.db")
    ints = counters(ipath, {"SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"}) if os.path.exists(ipath) else {}
    for k in sorted(set(dur) | set(fetch)):
        if k.startswith("void at::") or k.startswith("__amd"):
            continue
        s = sq.get(k, {})
        d = dur.get(k, [])
        keep = None
        if s.get("GRBM_GUI_ACTIVE") and d:
            gui_d = by_dispatch(s["GRBM_GUI_ACTIVE"])
            n = min(len(gui_d), len(d))
            keep = {i for i in range(n) if d[i] > 0 and CLK_LO <= gui_d[i] / 8 / d[i] <= CLK_HI}
        r = {"dispatches": len(d)}
        if keep is not None and len(keep) < len(d):
            r["implausible_clock_dispatches"] = len(d) - len(keep)
        dk = [x for i, x in enumerate(d) if keep is None or i in keep]
        r["avg_ms"] = round(sum(dk) / len(dk) / 1e6, 4) if dk else None
        if keep is not None and not keep:
            res[k] = r  # no plausible dispatch: nothing derived from an overlapped duration
            continue
        if "_res" in fetch.get(k, {}):
            vg, ag, scr = fetch[k]["_res"][0][1]
            r.update({"vgpr": vg, "agpr": ag, "scratch_bytes_per_lane": scr})
        if fetch.get(k, {}).get("FETCH_SIZE"):
            kb = per_dispatch(fetch[k]["FETCH_SIZE"], keep)
            r["fetch_bytes_raw"] = round(kb * 1024)
            r["fetch_bytes_x2"] = round(kb * 2048)
        if write.get(k, {}).get("WRITE_SIZE"):
            r["write_bytes"] = round(per_dispatch(write[k]["WRITE_SIZE"], keep) * 1024)
        if s.get("SQ_INSTS_VALU"):
            r["sq_insts_valu"] = per_dispatch(s["SQ_INSTS_VALU"], keep)
            r["sq_waves"] = per_dispatch(s["SQ_WAVES"], keep)
            wcyc = per_dispatch(s["SQ_WAVE_CYCLES"], keep) if s.get("SQ_WAVE_CYCLES") else None
            gui = per_dispatch(s["GRBM_GUI_ACTIVE"], keep) if s.get("GRBM_GUI_ACTIVE") else None
            if gui:
                # GRBM_GUI_ACTIVE sums the 8 XCDs' clocks; each of the 1024 SIMDs issues at most one
                # wave-instruction per cycle: VALU wave-instructions per SIMD per cycle
                r["valu_issue_per_simd_cycle"] = round(r["sq_insts_valu"] / (1024 * gui / 8), 4)
                r["gpu_cycles_per_dispatch"] = round(gui / 8)
                if r.get("avg_ms"):  # effective clock of the profiled run (MI355X_MICROARCH.md, DVFS)
                    r["profiled_clock_ghz"] = round(gui / 8 / (r["avg_ms"] * 1e6), 3)
            if wcyc and gui:
                # achieved occupancy: SQ_WAVE_CYCLES sums every resident wave's lifetime in quad-cycles
                # (MI355X_MICROARCH.md, cycle constants), so x 4 over the 1,024 SIMDs' cycles = the mean
                # number of resident waves per SIMD over the dispatch
                r["mean_waves_per_simd"] = round(wcyc * 4 / (1024 * gui / 8), 3)
            if wcyc:  # where the waves' cycles went (disjoint buckets, quad-cycle units)
                for key, name in (("SQ_WAIT_ANY", "wait_any_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_any_frac"),
                                  ("SQ_ACTIVE_INST_ANY", "active_inst_any_frac")):
                    if s.get(key):
                        r[name] = round(per_dispatch(s[key], keep) / wcyc, 4)
        i = ints.get(k, {})
        if i.get("SQ_INSTS_VALU_INT32"):
            r["sq_insts_valu_int32"] = per_dispatch(i["SQ_INSTS_VALU_INT32"], keep)
            r["sq_insts_valu_int64"] = per_dispatch(i.get("SQ_INSTS_VALU_INT64", []), keep)
        res[k] = r
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
