"""Diagnostic (GPU box): chunk roots of random bodies for a sweep of lengths, GPU vs the oracle
restatement; prints the lengths that disagree.  python tools/diag_chunk_sweep.py lo hi step [extra...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))
import gsv  # noqa: E402
from oracle import oracle as O  # noqa: E402

lo, hi, step = (int(x) for x in sys.argv[1:4])
ns = list(range(lo, hi, step)) + [int(x) for x in sys.argv[4:]]
rng = np.random.default_rng(1)
ctx = gsv.default_context()
bad = []
for k in range(0, len(ns), 64):
    part = ns[k:k + 64]
    bodies = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in part]
    out = ctx.chunk_root_batch(bodies)
    for n, b, r in zip(part, bodies, out):
        if bytes(r) != O.derive_sha_bytes(b):
            bad.append(n)
print("checked", len(ns), "bad", len(bad), bad[:200], flush=True)
