"""GPU parity: batched secp256k1 recovery (gsv_ecrecover_batch / gsv_sender_batch) vs the oracle
and the reference's golden vectors, bit-exact."""
import random

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
HALF_N = N_ORDER // 2


def test_ecrecover_golden(ctx):
    cases = golden("ecrecover.json")["cases"]
    msgs = np.array([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in cases])
    sigs = np.array([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in cases])
    pub, addr, st = ctx.ecrecover_batch(msgs, sigs, want_pub=True, want_addr=True)
    for i, c in enumerate(cases):
        want = {1: 0, 0: 4, -1: 3}[c["rc"]]
        assert st[i] == want, (i, c["note"], st[i])
        if c["rc"] == 1:
            assert bytes(pub[i]).hex() == c["pub"], c["note"]
        else:
            assert not pub[i].any()


def test_ecrecover_random_vs_oracle(ctx, oracle):
    rng = random.Random(21)
    n = 1500
    msgs = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 65), np.uint8)
    for i in range(n):
        m = bytes(rng.getrandbits(8) for _ in range(32))
        kind = i % 5
        if kind < 3:  # valid signature from the oracle signer
            key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
            k = rng.randrange(1, N_ORDER).to_bytes(32, "big")
            s = oracle.secp_sign(m, key, k)
        elif kind == 3:  # random r, s, recid
            s = (rng.randrange(1, N_ORDER).to_bytes(32, "big") + rng.randrange(1, N_ORDER).to_bytes(32, "big")
                 + bytes([rng.randrange(4)]))
        else:  # small / structured values
            r = rng.choice([1, 2, 3, 4, 5, 7, rng.randrange(1, 2**64)])
            s = r.to_bytes(32, "big") + rng.randrange(1, N_ORDER).to_bytes(32, "big") + bytes([rng.randrange(4)])
        msgs[i] = np.frombuffer(m, np.uint8)
        sigs[i] = np.frombuffer(s, np.uint8)
    pub, addr, st = ctx.ecrecover_batch(msgs, sigs, want_pub=True, want_addr=True)
    opub, ost = oracle.ecrecover_batch(msgs, sigs)
    assert (st == ost).all(), np.nonzero(st != ost)[0][:10]
    assert (pub == opub).all()
    ok = st == 0
    for i in np.nonzero(ok)[0][:200]:
        assert bytes(addr[i]) == oracle.keccak256(bytes(pub[i, 1:]))[12:]


def test_ecrecover_matches_reference_build(ctx, oracle):
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref not built on this machine")
    import ctypes
    rng = random.Random(33)
    n = 256
    msgs = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 65), np.uint8)
    for i in range(n):
        key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
        m = bytes(rng.getrandbits(8) for _ in range(32))
        sig = ctypes.create_string_buffer(65)
        R.gsvref_sign(sig, m, key)
        msgs[i] = np.frombuffer(m, np.uint8)
        sigs[i] = np.frombuffer(sig.raw, np.uint8)
    pub, _, st = ctx.ecrecover_batch(msgs, sigs)
    rpub = np.zeros((n, 65), np.uint8)
    ok = R.gsvref_ecrecover_many(rpub.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                 sigs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                 msgs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), n)
    assert ok == n and (st == 0).all() and (pub == rpub).all()


def test_synth_sign_roundtrip_and_oracle(ctx, oracle):
    n = 4096
    msg, sig, pub, addr = ctx.synth_sign(seed=12345, n=n)
    rpub, raddr, st = ctx.ecrecover_batch(msg, sig, want_pub=True, want_addr=True)
    assert (st == 0).all()
    assert (rpub == pub).all() and (raddr == addr).all()
    # the GPU signer is bit-exact with the oracle signer on a sample
    import struct
    for i in [0, 1, 2, 777, 4095]:
        def derive(tag):
            return oracle.keccak256(struct.pack("<QQ", 12345, i) + tag)
        d = int.from_bytes(derive(b"key"), "big") % N_ORDER or 1
        k = int.from_bytes(derive(b"nce"), "big") % N_ORDER or 1
        m = derive(b"msg")
        assert bytes(msg[i]) == m
        want = oracle.secp_sign(m, d.to_bytes(32, "big"), k.to_bytes(32, "big"))
        assert bytes(sig[i]) == want
        assert bytes(pub[i]) == oracle.secp_pubkey(d.to_bytes(32, "big"))


def test_sender_batch_recover_plain(ctx, oracle):
    # recoverPlain + ValidateSignatureValues (core/types/transaction_signing.go:222-247)
    rng = random.Random(8)
    rows = []
    for i in range(300):
        key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
        m = bytes(rng.getrandbits(8) for _ in range(32))
        s = oracle.secp_sign(m, key, rng.randrange(1, N_ORDER).to_bytes(32, "big"))
        r_, s_, v_ = int.from_bytes(s[:32], "big"), int.from_bytes(s[32:64], "big"), s[64] + 27
        vbig = 0
        kind = i % 10
        if kind == 1:
            s_ = N_ORDER - s_  # high s: homestead rejects, frontier accepts (recovers other key)
            v_ ^= 1
        elif kind == 2:
            v_ = 29  # V = 2 -> invalid
        elif kind == 3:
            vbig = 1
        elif kind == 4:
            r_ = 0
        elif kind == 5:
            s_ = N_ORDER
        elif kind == 6:
            v_ = 3  # byte(3 - 27) wraps -> invalid
        rows.append((m, r_, s_, v_, vbig))
    n = len(rows)
    H = np.array([np.frombuffer(m, np.uint8) for m, *_ in rows])
    R_ = np.array([np.frombuffer(r.to_bytes(32, "big"), np.uint8) for _, r, *_ in rows])
    S_ = np.array([np.frombuffer(s.to_bytes(32, "big"), np.uint8) for _, _, s, *_ in rows])
    V = np.array([v for *_, v, _ in rows], np.uint64)
    VB = np.array([b for *_, b in rows], np.uint8)
    for homestead in (True, False):
        addr, st = ctx.sender_batch(H, R_, S_, V, VB, homestead)
        import ctypes
        for i, (m, r_, s_, v_, vb) in enumerate(rows):
            out = ctypes.create_string_buffer(20)
            vbytes = v_.to_bytes(2, "big") if not vb else b"\x01\x00\x00"
            want = oracle.lib().oracle_recover_plain(out, m, r_.to_bytes(32, "big"), 32, s_.to_bytes(32, "big"),
                                                     32, vbytes, len(vbytes), 1 if homestead else 0)
            assert st[i] == want, (i, homestead)
            if want == 0:
                assert bytes(addr[i]) == out.raw


def test_ecrecover_large_differential_vs_oracle(ctx, oracle):
    """131,072 signatures through the batch API against the oracle restatement (16 host threads), bit
    for bit: GPU-signed valid signatures, the same with recid flipped (a different, valid point or a
    non-residue), s -> n - s (high s: ecrecover accepts it, the key changes), r and s replaced by random
    values below n / at n and above / zero, recids 0..3 and out of range, and messages of all zeros and
    ones.  Status and public key must match for every item."""
    n = 1 << 17
    msg, sig, _, _ = ctx.synth_sign(20251018, n, want_pub=False, want_addr=False)
    rng = np.random.default_rng(77)
    kind = rng.integers(0, 8, n)
    sig = sig.copy()
    msg = msg.copy()
    be = lambda v: np.frombuffer(int(v).to_bytes(32, "big"), np.uint8)
    nb = be(N_ORDER)
    for i in np.nonzero(kind == 1)[0]:  # recid flipped
        sig[i, 64] ^= 1
    for i in np.nonzero(kind == 2)[0]:  # high s
        s = int.from_bytes(sig[i, 32:64].tobytes(), "big")
        sig[i, 32:64] = be(N_ORDER - s)
    idx = np.nonzero(kind == 3)[0]  # random r, s below 2^256, recid 0..3
    sig[idx, :64] = rng.integers(0, 256, (idx.size, 64), dtype=np.uint8)
    sig[idx, 64] = rng.integers(0, 4, idx.size)
    for j, i in enumerate(np.nonzero(kind == 4)[0]):  # r or s at the edges: 0, n, n + 1, 2^256 - 1
        edge = [be(0), nb, be(N_ORDER + 1), np.full(32, 255, np.uint8)][j % 4]
        if j % 2:
            sig[i, :32] = edge
        else:
            sig[i, 32:64] = edge
    idx = np.nonzero(kind == 5)[0]  # recid out of range
    sig[idx, 64] = rng.choice(np.array([4, 5, 27, 28, 255], np.uint8), idx.size)
    idx = np.nonzero(kind == 6)[0]  # the message replaced (valid r, s: another key, same status rules)
    msg[idx] = rng.integers(0, 256, (idx.size, 32), dtype=np.uint8)
    idx = np.nonzero(kind == 7)[0]
    msg[idx[::2]] = 0
    msg[idx[1::2]] = 255
    pub, _, st = ctx.ecrecover_batch(msg, sig, want_pub=True, want_addr=False)
    opub, ost = oracle.ecrecover_batch(msg, sig, threads=16)
    bad = np.nonzero(st != ost)[0]
    assert bad.size == 0, [(int(i), int(kind[i]), int(st[i]), int(ost[i])) for i in bad[:10]]
    assert (pub == opub).all()
    # every class produced what it should: valid ones mostly valid, out-of-range recids all rejected
    assert (st[kind == 0] == 0).all() and (st[kind == 5] != 0).all()
    assert len(set(st.tolist())) >= 3
