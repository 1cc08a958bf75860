"""GPU parity: batched Keccak-256 (gsv_keccak256_batch) vs the golden vectors and the oracle."""
import random

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def test_keccak256_golden(ctx):
    vs = golden("keccak.json")["keccak256"]
    out = ctx.keccak256_batch([bytes.fromhex(v["msg"]) for v in vs])
    for i, v in enumerate(vs):
        assert bytes(out[i]).hex() == v["digest"], v["source"]


def test_keccak256_ragged_vs_oracle(ctx, oracle):
    rng = random.Random(3)
    msgs = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 7, 8, 9, 64, 135, 136, 137, 271, 272,
                                                                rng.randrange(0, 2000)])))
            for _ in range(700)]
    out = ctx.keccak256_batch(msgs)
    for i, m in enumerate(msgs):
        assert bytes(out[i]) == oracle.keccak256(m)


def test_keccak256_empty_batch(ctx):
    assert ctx.keccak256_batch([]).shape == (0, 32)
