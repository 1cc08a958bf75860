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


def _dev_hash(ctx, msgs, shift):
    """keccak256_batch_dev over the messages packed back to back starting `shift` bytes into the buffer
    (a misaligned base pointer: the LDS staging rounds the workgroup's span to 16-byte chunks)"""
    import torch
    flat = b"".join(msgs)
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    buf = torch.zeros(len(flat) + shift + 64, dtype=torch.uint8, device="cuda")
    buf[shift:shift + len(flat)] = torch.from_numpy(np.frombuffer(flat, np.uint8).copy()).cuda()
    data = buf[shift:]
    out = torch.empty((len(msgs), 32), dtype=torch.uint8, device="cuda")
    ctx.keccak256_batch_dev(data, torch.from_numpy(off).cuda(), out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("shift", [0, 1, 3, 13])
def test_keccak256_tx_sized_staged(ctx, oracle, shift):
    """100-160-byte messages (the bench's tx-string shape): every workgroup's 256 messages fit the LDS
    staging buffer, so each lane assembles its blocks from LDS; any base alignment."""
    rng = np.random.default_rng(11 + shift)
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(100, 161, 1500)]
    out = _dev_hash(ctx, msgs, shift)
    for i, m in enumerate(msgs):
        assert bytes(out[i]) == oracle.keccak256(m), i


def test_keccak256_staged_and_direct_workgroups(ctx, oracle):
    """Workgroups whose span exceeds the 36 KiB staging buffer (a long message among them, or many
    medium ones) read straight from HBM; the others stage.  Spans just below and above the limit, a
    message crossing the limit, empty messages and a 100 KB message in one batch."""
    rng = np.random.default_rng(5)
    lens = []
    lens += list(rng.integers(100, 161, 256))       # wg 0: staged
    lens += [40000] + list(rng.integers(0, 50, 255))  # wg 1: a long message -> direct
    lens += [144] * 255 + [36864 - 144 * 255 - 16]    # wg 2: span just below 36 KiB (+ alignment slack)
    lens += [144] * 255 + [36864 - 144 * 255 + 40]    # wg 3: just above -> direct
    lens += [0] * 200 + [100000] + [1] * 55           # wg 4: empty messages and one 100 KB message
    lens += list(rng.integers(130, 140, 300))          # wg 5 + a partial wg 6
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    for shift in (0, 7):
        out = _dev_hash(ctx, msgs, shift)
        for i, m in enumerate(msgs):
            assert bytes(out[i]) == oracle.keccak256(m), (shift, i, len(m))


def test_keccak256_large_ragged_vs_oracle(ctx, oracle):
    """40,000 messages of uniformly random length 0..1,100 bytes (zero to nine rate blocks, every
    padding position) hashed in one batch, each against the oracle; the theta form of r05 (one
    three-input XOR per word) runs in every one of them."""
    rng = np.random.default_rng(1018)
    lens = rng.integers(0, 1101, 40000)
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    msgs, o = [], 0
    for n in lens:
        msgs.append(blob[o:o + int(n)])
        o += int(n)
    out = ctx.keccak256_batch(msgs)
    bad = [i for i, m in enumerate(msgs) if bytes(out[i]) != oracle.keccak256(m)]
    assert not bad, bad[:10]
