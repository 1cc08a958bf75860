"""A/B sweep of the pairing check's pairs-per-Miller-lane split (GSV_BN_PAIRS_PER_LANE) and
final-exponentiation layout (GSV_BN_FINAL3) at the
configs[4] batch per GPU for N = 1, 2, 4, 8 ranks (65,536 / N checks).  Every run checks the
verdicts against the generator's constructed truth.  Run on the GPU box from the repo root:
    python tools/pairing_sweep.py [checks ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))

import numpy as np
import torch

import gsv
from gsv import _lib


def run(ctx, n, k, f3=None, reps=2, m2=None):
    if k:
        os.environ["GSV_BN_PAIRS_PER_LANE"] = str(k)
    else:
        os.environ.pop("GSV_BN_PAIRS_PER_LANE", None)
    if f3 is not None:
        os.environ["GSV_BN_FINAL3"] = str(f3)
    else:
        os.environ.pop("GSV_BN_FINAL3", None)
    if m2 is not None:
        os.environ["GSV_BN_MILLER2"] = str(m2)
    else:
        os.environ.pop("GSV_BN_MILLER2", None)
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    pexp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    pver = torch.empty((n,), dtype=torch.uint8, device="cuda")
    src = os.environ.get("SWEEP_INPUT")  # A/B on fixed bytes: SWEEP_INPUT=path[.npz] (made on first use)
    if src and os.path.exists(src):
        z = np.load(src)
        pin.copy_(torch.from_numpy(z["pin"][:n]).to(pin.device))
        pexp.copy_(torch.from_numpy(z["pexp"][:n]).to(pexp.device))
    else:
        ctx.bn256_synth_checks_dev(5000, pin, pexp)
        torch.cuda.synchronize()  # the generator runs on the context's stream
        if src:
            np.savez(src, pin=pin.cpu().numpy(), pexp=pexp.cpu().numpy())
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.pairing_check_batch_dev(pin, off, pver)
    torch.cuda.synchronize()
    assert torch.equal(pver, pexp), "verdicts differ from the constructed truth"
    ctx.reset_timing()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.pairing_check_batch_dev(pin, off, pver)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ctx.set_timing(False)
    ks = [ctx.kernel_time(k)[0] / reps for k in (_lib.K_BN_PREPARE, _lib.K_PAIRING, _lib.K_BN_FINAL)]
    return dt, ks


CASES = ((0, None, None), (1, None, None), (2, None, None), (4, None, None), (0, 0, None), (0, 1, None),
         (0, None, 0), (0, None, 1), (2, None, 1))
if os.environ.get("SWEEP_CASES"):  # e.g. "4,,1;2,,1" = k,final3,miller2 (empty = auto)
    CASES = tuple(tuple(int(x) if x else (0 if i == 0 else None) for i, x in enumerate(c.split(",")))
                  for c in os.environ["SWEEP_CASES"].split(";"))


_STREAMS = []


def run_pipelined(ctx, n, depth, steps=None, streams=None):
    """n checks per batch, consecutive batches over `depth` streams (gsv_ctx_set_pipeline_depth)"""
    steps = steps or int(os.environ.get("SWEEP_STEPS", "12"))
    if not os.environ.get("SWEEP_KEEP_LAYOUT"):  # else the GSV_BN_* overrides in the environment apply
        for v in ("GSV_BN_PAIRS_PER_LANE", "GSV_BN_FINAL3", "GSV_BN_MILLER2"):
            os.environ.pop(v, None)
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    pexp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(5000, pin, pexp)
    torch.cuda.synchronize()
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.set_pipeline_depth(depth)
    ctx.pairing_prepare(off)
    ctx.set_pipeline_depth(1)
    global _STREAMS
    if streams is not None:
        ss = streams
    elif os.environ.get("SWEEP_REUSE_STREAMS") and len(_STREAMS) >= depth:
        ss = _STREAMS[:depth]  # the same HIP streams as the previous run
    elif os.environ.get("SWEEP_TORCH_STREAMS"):  # torch's pool streams (may share a hardware queue)
        ss = [torch.cuda.Stream() for _ in range(depth)]
        _STREAMS = ss
    else:  # streams on hardware queues of their own (gsv_stream_create), as bench.py
        ss = ctx.pipeline_streams(depth)
        _STREAMS = ss
    pv = [torch.empty((n,), dtype=torch.uint8, device="cuda") for _ in range(depth)]
    for i in range(depth):
        ctx.pairing_check_batch_dev(pin, off, pv[i], stream=ss[i], prepare=False)
    torch.cuda.synchronize()
    assert all(torch.equal(v, pexp) for v in pv), "verdicts differ from the constructed truth"
    # warm-up at full depth before timing (a fresh process's first batches read ~1.4x slow: clocks and
    # first-use costs; r04/r05 sweeps that timed the first depth of a process carried that artifact)
    for i in range(4 * depth):
        ctx.pairing_check_batch_dev(pin, off, pv[i % depth], stream=ss[i % depth], prepare=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        ctx.pairing_check_batch_dev(pin, off, pv[i % depth], stream=ss[i % depth], prepare=False)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    if streams is None and not os.environ.get("SWEEP_REUSE_STREAMS"):
        # a process's dedicated queues stay few: dozens of them (idle ones included) oversubscribe the
        # hardware scheduler and every run slows (r05: 8,192 checks three deep 8.6 vs 3.8 ms per batch)
        ctx.destroy_streams(ss)
        _STREAMS = []
    return dt


def preheat(ctx, seconds=1.5):
    """GPU-busy for a while before anything is timed (SWEEP_PREHEAT=1): the first pipelined run of a
    process read ~1.5x slow even after its own warm-up batches (profiles/r05/ab/pipe_rep_8192.txt)."""
    n = 65536
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(5000, pin, None)
    torch.cuda.synchronize()
    off = np.arange(n + 1, dtype=np.uint64) * 768
    pv = torch.empty((n,), dtype=torch.uint8, device="cuda")
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ctx.pairing_check_batch_dev(pin, off, pv)
        torch.cuda.synchronize()


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [65536, 32768, 16384, 8192]
    ctx = gsv.default_context()
    if os.environ.get("SWEEP_PREHEAT"):
        preheat(ctx)
    if os.environ.get("SWEEP_STREAM_SETS"):  # e.g. "0,1,2;3,4,5": pipelines over chosen pool streams
        owned = bool(os.environ.get("SWEEP_CUMASK"))
        if owned:  # streams on queues of their own (gsv_stream_create: a CU mask of every CU), at most 8
            pool = ctx.pipeline_streams(int(os.environ["SWEEP_CUMASK"]))
        else:
            pool = [torch.cuda.Stream() for _ in range(16)]
        print("pool streams:", " ".join(hex(s_.cuda_stream) for s_ in pool), flush=True)
        for n in sizes:
            for st in os.environ["SWEEP_STREAM_SETS"].split(";"):
                ix = [int(x) for x in st.split(",")]
                dt = run_pipelined(ctx, n, len(ix), streams=[pool[i] for i in ix])
                print(f"streams {st:>10} checks {n:6d} depth {len(ix)}: {dt * 1e3:8.2f} ms per batch", flush=True)
        torch.cuda.synchronize()
        if owned:
            ctx.destroy_streams(pool)
        return
    if os.environ.get("SWEEP_PIPELINE"):  # e.g. "1,2,3": pipeline depths at auto layout
        for n in sizes:
            for d in (int(x) for x in os.environ["SWEEP_PIPELINE"].split(",")):
                dt = run_pipelined(ctx, n, d)
                print(f"checks {n:6d} pipeline depth {d}: {dt * 1e3:8.2f} ms per batch  {n / dt / 1e6:.3f} M checks/s",
                      flush=True)
        return
    for n in sizes:
        for k, f3, m2 in CASES:
            dt, ks = run(ctx, n, k, f3, m2=m2)
            print(f"checks {n:6d} k {k or 'auto':>4} final3 {'auto' if f3 is None else f3:>4} "
                  f"miller2 {'auto' if m2 is None else m2:>4}: {dt * 1e3:8.2f} ms  "
                  f"{n / dt / 1e6:.3f} M checks/s  prepare/miller/final {ks[0]:.2f}/{ks[1]:.2f}/{ks[2]:.2f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
