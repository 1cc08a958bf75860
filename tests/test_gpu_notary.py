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


def _signed_tx(oracle, key, nonce, data, chain_id, eip155=True, want_zero=None):
    """An EIP-155 (or unprotected Homestead) transaction signed with `key`; want_zero = "r" / "s" retries
    the signing nonce until that value's top byte is zero (a 31-byte or shorter RLP string)."""
    to = bytes(range(1, 21))
    fields = (oracle.rlp_uint(nonce) + oracle.rlp_uint(20 * 10 ** 9) + oracle.rlp_uint(21000 + len(data)) +
              oracle.rlp_string(to) + oracle.rlp_uint(10 ** 18 + nonce) + oracle.rlp_string(data))
    pre = fields + (oracle.rlp_uint(chain_id) + b"\x80\x80" if eip155 else b"")
    h = oracle.keccak256(oracle.rlp_list(pre))
    for k in range(1, 5000):
        sig = oracle.secp_sign(h, key, k.to_bytes(32, "big"))
        if want_zero is None or sig[0 if want_zero == "r" else 32] == 0:
            break
    else:
        raise AssertionError("no signature with the wanted leading zero")
    v = sig[64] + (35 + 2 * chain_id if eip155 else 27)
    r, s = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:64], "big")
    return oracle.rlp_list(fields + oracle.rlp_uint(v) + oracle.rlp_uint(r) + oracle.rlp_uint(s))


@pytest.mark.parametrize("chain_id", [0, 1, 137, 2 ** 31 + 11, 2 ** 63 + 5, 2 ** 100 + 7])
def test_notary_preimage_shapes(ctx, oracle, chain_id):
    """The sighash preimage and R / S are gathered as little-endian dwords through the chunk map
    (notary.hip BlobView::dword, PreStream::dword, item_limb): data fields of 0-1,100 bytes (list
    headers of one to three bytes, preimages of one to nine rate blocks, every chunk phase), chain ids
    whose rlp suffix is 3 to 16 bytes (chain id 0 included; V above 64 bits takes v_big_path), unprotected transactions in
    the same body, and R or S with a zero top byte (31-byte strings).  Statuses and senders against the
    oracle's types.Sender, and every sender against the signing key's address."""
    key = bytes.fromhex("4c0883a69102937d6231471b5dbb6204fe5129617082792ae468d01a3f362318")
    pub = oracle.secp_pubkey(key)
    addr = oracle.keccak256(pub[1:])[12:]
    rng = random.Random(chain_id % 1000)
    txs = []
    for i, n in enumerate([0, 1, 54, 55, 56, 57, 120, 135, 136, 137, 250, 400, 1100]):
        txs.append(_signed_tx(oracle, key, i, bytes(rng.getrandbits(8) for _ in range(n)), chain_id))
    txs.append(_signed_tx(oracle, key, 50, b"\x01\x02", chain_id, eip155=False))
    txs.append(_signed_tx(oracle, key, 51, bytes(200), chain_id, eip155=False))
    txs.append(_signed_tx(oracle, key, 52, b"", chain_id, want_zero="r"))
    txs.append(_signed_tx(oracle, key, 53, bytes(77), chain_id, want_zero="s"))
    for pad in range(1, 4):  # shift every later transaction's chunk phase
        txs.append(_signed_tx(oracle, key, 60 + pad, bytes(pad * 9), chain_id))
    body = oracle.blob_serialize(txs)
    _, ntx, _, senders, status = _check(ctx, oracle, [body], chain_id, 0, 64)
    assert ntx[0] == len(txs)
    assert (status[0, :len(txs)] == ST_OK).all(), status[0, :len(txs)]
    assert all(bytes(senders[0, t]) == addr for t in range(len(txs)))
