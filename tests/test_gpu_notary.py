"""GPU parity: notary validation of collation bodies (gsv_notary_validate_shards) — blob codec,
RLP tx decode, Sender recovery and chunk root on the GPU — against the CPU oracle
(oracle_blob_deserialize + oracle_tx_sender + oracle_derive_sha_bytes) and the golden tx vectors
(core/types/transaction_signing_test.go:74-101, transaction_test.go:88-125)."""
import random

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu

ST_OK, ST_INVALID_SIG, ST_INVALID_CHAIN_ID, ST_RECOVER_FAILED, ST_BAD_RLP = 0, 5, 6, 4, 8


def _oracle_expect(oracle, body: bytes, chain_id: int, signer: int, max_txs: int):
    blobs = oracle.blob_deserialize(body)
    st = np.full(max_txs, ST_BAD_RLP, np.uint8)
    snd = np.zeros((max_txs, 20), np.uint8)
    for t, (rlp, _skip) in enumerate(blobs[:max_txs]):
        s, a = oracle.tx_sender(rlp, chain_id, signer)
        st[t] = s
        if s == 0:
            snd[t] = np.frombuffer(a, np.uint8)
    bm = np.zeros((max_txs + 7) // 8, np.uint8)
    for t in range(min(len(blobs), max_txs)):
        if st[t] == 0:
            bm[t // 8] |= 1 << (t % 8)
    return len(blobs), st, snd, bm


def _check(ctx, oracle, bodies, chain_id=1, signer=0, max_txs=64):
    roots, ntx, bitmap, senders, status = ctx.notary_validate_shards(bodies, chain_id, signer, max_txs)
    for i, body in enumerate(bodies):
        n, st, snd, bm = _oracle_expect(oracle, body, chain_id, signer, max_txs)
        assert ntx[i] == n, i
        k = min(n, max_txs)
        assert (status[i, :k] == st[:k]).all(), (i, status[i, :k], st[:k])
        assert (senders[i, :k] == snd[:k]).all(), i
        assert (bitmap[i] == bm).all(), i
        assert bytes(roots[i]) == oracle.derive_sha_bytes(body), i
    return roots, ntx, bitmap, senders, status


def test_notary_golden_txs(ctx, oracle):
    vec = golden("tx.json")
    e155 = [bytes.fromhex(v["rlp"]) for v in vec["eip155_chain1"]]
    home = [bytes.fromhex(v["rlp"]) for v in vec["homestead"]]
    body = oracle.blob_serialize(e155 + home, skip_evm=[i % 2 for i in range(len(e155) + len(home))])
    roots, ntx, bitmap, senders, status = _check(ctx, oracle, [body], 1, 0, 32)
    for t, v in enumerate(vec["eip155_chain1"]):
        assert status[0, t] == ST_OK and bytes(senders[0, t]).hex() == v["addr"]
    # Homestead / Frontier signers over the same body
    _check(ctx, oracle, [body], 1, 1, 32)
    _check(ctx, oracle, [body], 1, 2, 32)
    # a different chain id: protected txs fail with ErrInvalidChainId
    _, _, _, _, st = _check(ctx, oracle, [body], 5, 0, 32)
    assert (st[0, :len(e155)] == ST_INVALID_CHAIN_ID).all()


def test_notary_edge_bodies(ctx, oracle):
    rng = random.Random(9)
    e155 = [bytes.fromhex(v["rlp"]) for v in golden("tx.json")["eip155_chain1"]]
    bodies = [
        b"",                                                   # empty body
        bytes(32 * 5),                                         # only non-terminal chunks: no blobs
        oracle.blob_serialize(e155[:3]) + bytes(17),           # trailing partial chunk ignored
        oracle.blob_serialize([b"\x01", b"\xc0", b"\x80"]),    # tiny blobs, not transactions
        oracle.blob_serialize([bytes(rng.getrandbits(8) for _ in range(n)) for n in (5, 40, 90, 200)]),
    ]
    # corrupted transactions: flip bytes inside RLP headers / fields
    for k in range(6):
        tx = bytearray(rng.choice(e155))
        tx[rng.randrange(len(tx))] ^= 1 << rng.randrange(8)
        bodies.append(oracle.blob_serialize([bytes(tx)] + e155[:2]))
    # non-canonical encodings: leading zero in nonce, long form for a short string
    t0 = e155[0]
    bodies.append(oracle.blob_serialize([t0[:2] + b"\x81\x00" + t0[3:]]))
    _check(ctx, oracle, bodies, 1, 0, 16)


def test_notary_synthetic_shards(ctx, oracle):
    import torch
    n_sh, per = 3, 256
    bodies_t = torch.empty((n_sh * per * 128,), dtype=torch.uint8, device="cuda")
    exp_st = torch.empty((n_sh * per,), dtype=torch.uint8, device="cuda")
    exp_snd = torch.empty((n_sh * per, 20), dtype=torch.uint8, device="cuda")
    ctx.notary_synth_dev(42, 7, n_sh, per, bodies_t, exp_st, exp_snd)
    torch.cuda.synchronize()
    flat = bodies_t.cpu().numpy()
    bodies = [flat[i * per * 128:(i + 1) * per * 128].tobytes() for i in range(n_sh)]
    roots, ntx, bitmap, senders, status = _check(ctx, oracle, bodies, 1, 0, per)
    es = exp_st.cpu().numpy().reshape(n_sh, per)
    assert (status == es).all()
    # generator classes (gi / 128) % 4 with gi = shard * per + j: class 3 flips the recid, a valid
    # signature of another key (status OK, sender != the signer the generator expects)
    gi = (np.arange(7, 7 + n_sh)[:, None] * per + np.arange(per)[None, :])
    flip = (gi % 128 == 127) & ((gi // 128) % 4 == 3)
    assert flip.any()
    same = (senders == exp_snd.cpu().numpy().reshape(n_sh, per, 20)).all(axis=2)
    assert same[~flip].all() and not same[flip].any()
    assert (es == ST_OK).sum() == n_sh * per - n_sh * (per // 128) + flip.sum()
    # the device-resident entry point gives the same records
    h_off = np.arange(n_sh + 1, dtype=np.uint64) * per * 128
    r_t = torch.empty((n_sh, 32), dtype=torch.uint8, device="cuda")
    n_t = torch.empty((n_sh,), dtype=torch.int32, device="cuda")
    b_t = torch.empty((n_sh, per // 8), dtype=torch.uint8, device="cuda")
    ctx.notary_validate_shards_dev(bodies_t, h_off, r_t, n_t, b_t, max_txs=per)
    torch.cuda.synchronize()
    assert (r_t.cpu().numpy() == roots).all() and (b_t.cpu().numpy() == bitmap).all()
    assert (n_t.cpu().numpy() == per).all()


def test_notary_full_body_invalid_classes(ctx):
    """One full 2^20-byte shard (8,192 txs): the generator's expected statuses at full size,
    all three invalid classes present, ntx == 8192."""
    import torch
    per = 8192
    bodies_t = torch.empty((per * 128,), dtype=torch.uint8, device="cuda")
    exp_st = torch.empty((per,), dtype=torch.uint8, device="cuda")
    ctx.notary_synth_dev(5, 0, 1, per, bodies_t, exp_st, None)
    h_off = np.array([0, per * 128], np.uint64)
    r_t = torch.empty((1, 32), dtype=torch.uint8, device="cuda")
    n_t = torch.empty((1,), dtype=torch.int32, device="cuda")
    b_t = torch.empty((1, per // 8), dtype=torch.uint8, device="cuda")
    s_t = torch.empty((1, per), dtype=torch.uint8, device="cuda")
    ctx.notary_validate_shards_dev(bodies_t, h_off, r_t, n_t, b_t, None, s_t, max_txs=per)
    torch.cuda.synchronize()
    assert int(n_t[0]) == per
    assert torch.equal(s_t[0], exp_st)
    assert set(torch.unique(exp_st).tolist()) == {ST_OK, ST_INVALID_SIG, ST_INVALID_CHAIN_ID, ST_RECOVER_FAILED}


def test_tx_sender_batch_golden(ctx, oracle):
    vec = golden("tx.json")
    txs = [bytes.fromhex(v["rlp"]) for v in vec["eip155_chain1"]]
    addr, st = ctx.tx_sender_batch(txs, 1, 0)
    for i, v in enumerate(vec["eip155_chain1"]):
        assert st[i] == 0 and bytes(addr[i]).hex() == v["addr"]
    home = [bytes.fromhex(v["rlp"]) for v in vec["homestead"]]
    addr, st = ctx.tx_sender_batch(home, 1, 1)
    for i, v in enumerate(vec["homestead"]):
        s, a = oracle.tx_sender(home[i], 1, 1)
        assert st[i] == s and (s != 0 or bytes(addr[i]) == a)
