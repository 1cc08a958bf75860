"""k_ecrecover timing only (no parity check: for upper-bound variants whose results are wrong by
construction): 20 consecutive 2^20-signature batches on one stream after 6 warm-up batches, wall time
and HIP-event kernel time.  Library from GSV_LIB_PATH.  GPU box, repo root:
    python tools/ecr_time.py [label]"""
import sys
import time

import torch

sys.path.insert(0, "geth-sharding_amd")
import gsv  # noqa: E402
from gsv import _lib  # noqa: E402

N = 1 << 20
label = sys.argv[1] if len(sys.argv) > 1 else "main"
ctx = gsv.default_context()
dev = torch.device("cuda", 0)
msg = torch.empty((N, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((N, 65), dtype=torch.uint8, device=dev)
ctx.synth_sign_dev(1000, msg, sig)
p = torch.empty((N, 65), dtype=torch.uint8, device=dev)
a = torch.empty((N, 20), dtype=torch.uint8, device=dev)
s = torch.empty((N,), dtype=torch.uint8, device=dev)
st = torch.cuda.Stream()
torch.cuda.synchronize()
for _ in range(6):
    ctx.ecrecover_batch_dev(msg, sig, p, a, s, stream=st)
torch.cuda.synchronize()
ctx.reset_timing()
ctx.set_timing(True)
t0 = time.perf_counter()
for _ in range(20):
    ctx.ecrecover_batch_dev(msg, sig, p, a, s, stream=st)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
ctx.set_timing(False)
k_ms, k_n = ctx.kernel_time(_lib.K_ECRECOVER)
print(f"{label:>10}: {N / dt / 1e6:.2f} M recoveries/s  kernel {k_ms / max(k_n, 1):.3f} ms  "
      f"status-0 lanes {int((s == 0).sum())}", flush=True)
