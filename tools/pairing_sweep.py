"""A/B sweep of the pairing check's pairs-per-Miller-lane split (GSV_BN_PAIRS_PER_LANE) at the
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


def run(ctx, n, k, reps=2):
    if k:
        os.environ["GSV_BN_PAIRS_PER_LANE"] = str(k)
    else:
        os.environ.pop("GSV_BN_PAIRS_PER_LANE", None)
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    pexp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    pver = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(5000, pin, pexp)
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.pairing_check_batch_dev(pin, off, pver)
    torch.cuda.synchronize()
    assert torch.equal(pver, pexp), "verdicts differ from the constructed truth"
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.pairing_check_batch_dev(pin, off, pver)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return dt


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [65536, 32768, 16384, 8192]
    ctx = gsv.default_context()
    for n in sizes:
        for k in (0, 1, 2, 4):
            dt = run(ctx, n, k)
            print(f"checks {n:6d} k {k or 'auto':>4}: {dt * 1e3:8.2f} ms  {n / dt / 1e6:.3f} M checks/s", flush=True)


if __name__ == "__main__":
    main()
