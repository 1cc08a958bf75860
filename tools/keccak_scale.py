"""k_keccak256 throughput against batch size: 100-160-byte messages (the bench's tx-string shape),
400k (the bench leg) up to 6.4M per launch, kernel time from the library's HIP events.  Shows how
much of the bench leg's roofline gap is the short launch (ramp-up and tail) rather than the kernel."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))
import gsv  # noqa: E402
from gsv import _lib  # noqa: E402


def main():
    ctx = gsv.default_context()
    rng = np.random.default_rng(5)
    for n in [int(a) for a in sys.argv[1:]] or [400_000, 1_600_000, 6_400_000]:
        lens = rng.integers(100, 161, n)
        off = np.zeros(n + 1, np.int64)
        off[1:] = np.cumsum(lens)
        vals = torch.from_numpy(rng.integers(0, 256, int(off[-1]), dtype=np.uint8)).cuda()
        off_t = torch.from_numpy(off).cuda()
        out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ctx.keccak256_batch_dev(vals, off_t, out)
        torch.cuda.synchronize()
        ctx.reset_timing()
        ctx.set_timing(True)
        for _ in range(5):
            ctx.keccak256_batch_dev(vals, off_t, out)
        torch.cuda.synchronize()
        ctx.set_timing(False)
        ms, k = ctx.kernel_time(_lib.K_KECCAK)
        perms = int(np.sum(lens // 136 + 1))
        per = ms / k
        print(f"messages {n:9d}: {per:7.3f} ms per launch, {perms / per / 1e6:7.3f} G perm/s, "
              f"{n / per / 1e6:7.3f} G hashes/s", flush=True)


if __name__ == "__main__":
    main()
