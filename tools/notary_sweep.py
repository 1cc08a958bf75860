"""Notary step time against the shards one rank holds (configs[3] split over N = 8, 4, 2, 1 ranks: 13,
25, 50, 100 shards of 8,192 txs), one step at a time and with consecutive steps on `depth` streams
(gsv_ctx_set_pipeline_depth), through gsv_notary_validate_shards_dev (the partition call minus its
all-gather).  Every run checks the statuses against the construction.  GPU box, repo root:
    python tools/notary_sweep.py [shards ...]
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

TXS = 8192


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [13, 25, 50, 100]
    ctx = gsv.default_context()
    for n in sizes:
        st0 = torch.cuda.Stream()
        nb = torch.empty((n * TXS * 128,), dtype=torch.uint8, device="cuda")
        exp = torch.empty((n * TXS,), dtype=torch.uint8, device="cuda")
        ctx.notary_synth_dev(777, 0, n, TXS, nb, exp, None, stream=st0)
        off = np.arange(n + 1, dtype=np.uint64) * TXS * 128
        st0.synchronize()
        for depth in tuple(int(x) for x in os.environ.get("NOTARY_DEPTHS", "1,2,3").split(",")):
            ctx.set_pipeline_depth(depth)
            ctx.notary_prepare(off, max_txs=TXS)
            ctx.set_pipeline_depth(1)
            ss = ctx.pipeline_streams(depth)  # hardware queues of their own (gsv_stream_create)
            outs = [(torch.empty((n, 32), dtype=torch.uint8, device="cuda"),
                     torch.empty((n,), dtype=torch.int32, device="cuda"),
                     torch.empty((n, TXS // 8), dtype=torch.uint8, device="cuda"),
                     torch.empty((n, TXS), dtype=torch.uint8, device="cuda")) for _ in range(depth)]
            for i in range(depth):
                r, c, b, s = outs[i]
                ctx.notary_validate_shards_dev(nb, off, r, c, b, None, s, max_txs=TXS, stream=ss[i], prepare=False)
            torch.cuda.synchronize()
            for r, c, b, s in outs:
                assert torch.equal(s.view(-1), exp), "statuses differ from the construction"
            # 40 timed steps (r06; 12 through r05): a pipeline's fill and drain cost about one step's
            # latency per measurement, 0.1 ms per 13-shard step at 12 steps (profiles/r06/ab/notary_stagger_steps.txt)
            steps = int(os.environ.get("NOTARY_STEPS", "40"))
            t0 = time.perf_counter()
            for i in range(steps):
                r, c, b, _ = outs[i % depth]
                ctx.notary_validate_shards_dev(nb, off, r, c, b, None, None, max_txs=TXS, stream=ss[i % depth],
                                               prepare=False)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            kt = float("nan")
            if not os.environ.get("NOTARY_NO_TIMING"):  # a trace of the pipeline alone sets it
                ctx.reset_timing()
                ctx.set_timing(True)
                r, c, b, _ = outs[0]
                ctx.notary_validate_shards_dev(nb, off, r, c, b, None, None, max_txs=TXS, stream=ss[0], prepare=False)
                torch.cuda.synchronize()
                ctx.set_timing(False)
                kt = ctx.kernel_time(_lib.K_NOTARY)[0]
            ctx.destroy_streams(ss)
            print(f"shards {n:4d} depth {depth}: {dt * 1e3:7.3f} ms per step  {n / dt:9.1f} shards/s  "
                  f"tx kernels {kt:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
