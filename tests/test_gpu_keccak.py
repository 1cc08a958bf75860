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
def test_keccak256_tx_sized_any_alignment(ctx, oracle, shift):
    """100-160-byte messages (the bench's tx-string shape, one or two rate blocks): each lane reads its
    blocks as aligned dwords realigned with v_alignbyte (keccak.hip load_block), at any base alignment."""
    rng = np.random.default_rng(11 + shift)
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(100, 161, 1500)]
    out = _dev_hash(ctx, msgs, shift)
    for i, m in enumerate(msgs):
        assert bytes(out[i]) == oracle.keccak256(m), i


def test_keccak256_block_count_buckets_per_workgroup(ctx, oracle):
    """The kernel takes each 256-message workgroup's messages in block-count order (keccak_dev.cuh
    wg_bucket_order: buckets 0..7 blocks and 8+, the last one shared by every longer message): one long
    message among short ones, block counts at and past the last bucket (8 x 136 = 1,088 bytes and up),
    exact multiples of the rate (the padding block alone), empty messages, a 100 KB message, and a
    partial last workgroup, at two base alignments."""
    rng = np.random.default_rng(5)
    lens = []
    lens += list(rng.integers(100, 161, 256))                       # wg 0: one or two blocks
    lens += [40000] + list(rng.integers(0, 50, 255))                # wg 1: one long message
    lens += [136 * k for k in range(10)] * 25 + [1087, 1088, 1089, 1223, 1224, 1225]  # wg 2: rate multiples
    lens += [0] * 200 + [100000] + [1] * 55                         # wg 3: empty messages and 100 KB
    lens += list(rng.integers(130, 140, 300))                       # wg 4 + a partial wg 5
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


def test_keccak256_tail_block_reads_at_batch_end(ctx, oracle):
    """The final block is read as whole 16-byte groups (keccak.hip load_block_tail) when at least 16
    bytes of the batch follow the message; the bytes read past it (the next messages) are masked.  A wave
    holding a message that ends within 16 bytes of the batch's end reads dword by dword instead.  Here
    the batch ends on a 4 KB boundary of its allocation with 0xff bytes after it, and its last messages
    are 0-17 bytes long; the batch starts at every alignment 0-3."""
    import torch
    for shift in range(4):
        rng = np.random.default_rng(77)
        lens = [100 + shift] + list(rng.integers(100, 161, 700)) + list(range(18)) + [0, 0, 5]
        msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
        flat = np.frombuffer(b"".join(msgs), np.uint8).copy()
        off = np.zeros(len(msgs) + 1, np.int64)
        off[1:] = np.cumsum(lens)
        buf = torch.full((len(flat) + 3 * 4096,), 0xff, dtype=torch.uint8, device="cuda")
        end = ((buf.data_ptr() + len(flat) + 4096) // 4096) * 4096 - buf.data_ptr()  # page-aligned end
        start = end - len(flat)
        assert 0 <= start and end + 16 <= buf.numel()
        buf[start:end] = torch.from_numpy(flat).cuda()
        out = torch.empty((len(msgs), 32), dtype=torch.uint8, device="cuda")
        ctx.keccak256_batch_dev(buf[start:end], torch.from_numpy(off).cuda(), out)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        bad = [i for i, m in enumerate(msgs) if bytes(o[i]) != oracle.keccak256(m)]
        assert not bad, ((buf.data_ptr() + start) % 4, bad[:10])


@pytest.mark.parametrize("out_shift", [1, 4, 8])
def test_keccak256_unaligned_digest_output(ctx, oracle, out_shift):
    """Digests to an output buffer that is not 16-byte aligned (the kernels store two dwordx4 only when it
    is, bytes otherwise), across whole workgroups of messages with one to three rate blocks."""
    import torch
    rng = np.random.default_rng(31 + out_shift)
    lens = rng.integers(0, 400, 1300)
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    flat = np.frombuffer(b"".join(msgs), np.uint8).copy()
    off = np.zeros(len(msgs) + 1, np.int64)
    off[1:] = np.cumsum(lens)
    data = torch.zeros(len(flat) + 64, dtype=torch.uint8, device="cuda")
    data[:len(flat)] = torch.from_numpy(flat).cuda()
    big = torch.full((len(msgs) * 32 + 32,), 0xee, dtype=torch.uint8, device="cuda")
    out = big[out_shift:out_shift + len(msgs) * 32].view(len(msgs), 32)
    ctx.keccak256_batch_dev(data, torch.from_numpy(off).cuda(), out)
    torch.cuda.synchronize()
    o = big.cpu().numpy()
    assert (o[:out_shift] == 0xee).all() and (o[out_shift + len(msgs) * 32:] == 0xee).all()
    bad = [i for i, m in enumerate(msgs) if bytes(o[out_shift + 32 * i:out_shift + 32 * i + 32]) != oracle.keccak256(m)]
    assert not bad, bad[:10]
