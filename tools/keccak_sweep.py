"""The bench's Keccak leg workload (400,000 tx-sized strings of 100-160 bytes) timed alone: kernel time
on HIP events and wall time per batch at one and two batches in flight (dedicated queues), with the
outputs checked equal across runs.  Launch knobs come from the environment (GSV_KECCAK_BLOCK ...), so
run one process per variant.  GPU box, repo root:
    python tools/keccak_sweep.py [label]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))
sys.path.insert(0, ROOT)

import numpy as np
import torch

import gsv
from gsv import _lib
from bench import _tx_strings


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    ctx = gsv.default_context()
    nblk, ntx, lens, voff, vals_np = _tx_strings(0)
    vals = torch.from_numpy(vals_np).cuda()
    off = torch.from_numpy(voff.astype(np.int64)).cuda()
    n = nblk * ntx
    perms = int(np.sum(lens // 136 + 1))
    ref = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for depth in tuple(int(x) for x in os.environ.get("KECCAK_DEPTHS", "1,2").split(",")):
        ss = ctx.pipeline_streams(depth)
        outs = [ref if d == 0 else torch.empty_like(ref) for d in range(depth)]
        for i in range(4):
            ctx.keccak256_batch_dev(vals, off, outs[i % depth], stream=ss[i % depth])
        torch.cuda.synchronize()
        steps = 80
        t0 = time.perf_counter()
        for i in range(steps):
            ctx.keccak256_batch_dev(vals, off, outs[i % depth], stream=ss[i % depth])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        assert all(torch.equal(ref, o) for o in outs)
        ctx.reset_timing()
        ctx.set_timing(True)
        for _ in range(8):
            ctx.keccak256_batch_dev(vals, off, ref, stream=ss[0])
        torch.cuda.synchronize()
        ctx.set_timing(False)
        k_ms, k_n = ctx.kernel_time(_lib.K_KECCAK)
        ctx.destroy_streams(ss)
        print(f"{label:>12} depth {depth}: {dt * 1e3:.4f} ms per batch  {perms / dt / 1e9:.3f} G perm/s  "
              f"kernel {k_ms / max(k_n, 1):.4f} ms  digest {int(ref.to(torch.int64).sum())}", flush=True)


if __name__ == "__main__":
    main()
