"""tools/pmc_summary.py on synthetic rocprofv3 outputs (CPU): a dispatch whose trace duration is not its
own (it ran beside another kernel in the trace pass, so GRBM_GUI_ACTIVE / 8 / duration is no clock the
GPU can run at) is dropped from every per-dispatch figure (pmc_notary.json reported
"clocks" of 0.054 and 5.7 GHz)."""
import io
import json
import os
import sqlite3
import sys
from contextlib import redirect_stdout

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def _db(path, create, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    con = sqlite3.connect(path)
    con.execute(create)
    con.executemany("insert into " + create.split()[2] + " values (" + ",".join("?" * len(rows[0])) + ")", rows)
    con.commit()
    con.close()


def _counters(kernels):
    """counters_collection rows: per kernel, per dispatch, per counter one value split over two shader engines"""
    rows, disp = [], 0
    for name, per in kernels:
        for vals in per:
            disp += 1
            for cname, v in vals.items():
                rows += [(name, cname, v / 2, disp, 128, 0, 0), (name, cname, v / 2, disp, 128, 0, 0)]
    return rows


def test_overlapped_dispatches_are_dropped(tmp_path):
    import pmc_summary
    root = str(tmp_path)
    ms = 1_000_000  # ns
    # k_a: three dispatches of 1 ms; the second ran beside another kernel in the trace pass (20 ms)
    # k_b: every dispatch implausible (a tiny kernel whose counter window holds the dispatch overhead)
    trace = [("gsv::k_a(int)", 0, 1 * ms), ("gsv::k_a(int)", 5 * ms, 25 * ms), ("gsv::k_a(int)", 30 * ms, 31 * ms),
             ("gsv::k_b(int)", 40 * ms, 40 * ms + 1000)]
    _db(os.path.join(root, "trace", "run_results.db"), "create table kernels (name text, start int, end int)", trace)
    gui_a = 8 * 2.0e6  # 2.0 GHz over 1 ms, summed over the 8 XCDs
    sq = _counters([("gsv::k_a(int)", [{"GRBM_GUI_ACTIVE": gui_a, "SQ_INSTS_VALU": 1000.0, "SQ_WAVES": 64.0,
                                        "SQ_WAVE_CYCLES": 100.0}] * 3),
                    ("gsv::k_b(int)", [{"GRBM_GUI_ACTIVE": 8 * 50000.0, "SQ_INSTS_VALU": 10.0, "SQ_WAVES": 1.0,
                                        "SQ_WAVE_CYCLES": 1.0}])])
    cc = ("create table counters_collection (kernel_name text, counter_name text, value real, dispatch_id int, "
          "vgpr_count int, accum_vgpr_count int, scratch_size int)")
    _db(os.path.join(root, "sq", "run_results.db"), cc, sq)
    fetch = _counters([("gsv::k_a(int)", [{"FETCH_SIZE": 100.0}, {"FETCH_SIZE": 900.0}, {"FETCH_SIZE": 100.0}]),
                       ("gsv::k_b(int)", [{"FETCH_SIZE": 5.0}])])
    _db(os.path.join(root, "fetch", "run_results.db"), cc, fetch)
    write = _counters([("gsv::k_a(int)", [{"WRITE_SIZE": 10.0}] * 3), ("gsv::k_b(int)", [{"WRITE_SIZE": 1.0}])])
    _db(os.path.join(root, "write", "run_results.db"), cc, write)
    buf = io.StringIO()
    with redirect_stdout(buf):
        pmc_summary.main(root)
    d = json.loads(buf.getvalue())
    a, b = d["gsv::k_a"], d["gsv::k_b"]
    assert a["dispatches"] == 3 and a["implausible_clock_dispatches"] == 1
    assert a["avg_ms"] == 1.0                          # the 20 ms overlapped duration is not averaged in
    assert a["profiled_clock_ghz"] == 2.0
    assert a["fetch_bytes_raw"] == 100 * 1024          # the overlapped dispatch's counters are dropped too
    assert b["dispatches"] == 1 and b["implausible_clock_dispatches"] == 1
    assert b["avg_ms"] is None and "profiled_clock_ghz" not in b and "fetch_bytes_raw" not in b
