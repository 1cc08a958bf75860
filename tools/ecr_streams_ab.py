"""A/B: consecutive 2^20-signature ecrecover batches on one stream vs two dedicated-queue streams
(gsv_stream_create), timed over 20 batches after a warm-up; prints recoveries/s for each."""
import sys
import time

import torch

sys.path.insert(0, "geth-sharding_amd")
import gsv  # noqa: E402

N = 1 << 20
ctx = gsv.default_context()
dev = torch.device("cuda", 0)
msg = torch.empty((N, 32), dtype=torch.uint8, device=dev)
sig = torch.empty((N, 65), dtype=torch.uint8, device=dev)
ctx.synth_sign_dev(1000, msg, sig)
torch.cuda.synchronize()
outs = [(torch.empty((N, 65), dtype=torch.uint8, device=dev), torch.empty((N, 20), dtype=torch.uint8, device=dev),
         torch.empty((N,), dtype=torch.uint8, device=dev)) for _ in range(2)]


def run(streams, steps=20):
    for i in range(4):
        p, a, s = outs[i % len(streams) if len(streams) > 1 else 0]
        ctx.ecrecover_batch_dev(msg, sig, p, a, s, stream=streams[i % len(streams)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        p, a, s = outs[i % len(streams) if len(streams) > 1 else 0]
        ctx.ecrecover_batch_dev(msg, sig, p, a, s, stream=streams[i % len(streams)])
    torch.cuda.synchronize()
    return N * steps / (time.perf_counter() - t0)


for rep in range(3):
    one = ctx.pipeline_streams(1)
    r1 = run(one)
    ctx.destroy_streams(one)
    two = ctx.pipeline_streams(2)
    r2 = run(two)
    ctx.destroy_streams(two)
    assert torch.equal(outs[0][0], outs[1][0])
    print(f"rep {rep}: one stream {r1 / 1e6:.2f} M/s, two streams {r2 / 1e6:.2f} M/s", flush=True)
