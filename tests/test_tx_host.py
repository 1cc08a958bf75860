"""The batch types.Sender host decoder (geth-sharding_amd/csrc/tx_host.hip: strict RLP decode of
txdata and the signer's sighash preimage) against the oracle, on the reference's transaction
vectors and on ~20,000 malformed variants of them (truncations, byte flips, corrupted length
prefixes, inserted bytes).  tools/sanitize.sh runs this file under ASan/UBSan.  CPU-only.

Reference: core/types/transaction.go:55-70 (txdata), transaction_signing.go:72-247 (signers),
rlp/decode.go (canonical sizes / integers)."""
import ctypes
import random

import pytest

from conftest import build_native, golden

ST_OK, ST_INVALID_SIG, ST_INVALID_CHAIN_ID, ST_BAD_RLP = 0, 5, 6, 8


@pytest.fixture(scope="module")
def txh(tmp_path_factory):
    L = build_native("tx_host_harness.cpp", tmp_path_factory.mktemp("txh") / "tx_host.so")
    L.h_tx_prepare.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), ctypes.c_char_p,
                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint8),
                               ctypes.POINTER(ctypes.c_int)]
    return L


def prepare(L, rlp, chain_id, kind):
    cid = chain_id.to_bytes((chain_id.bit_length() + 7) // 8, "big") if chain_id else b""
    pre = ctypes.create_string_buffer(len(rlp) + 64)
    n, rs, v, vbig, hs = ctypes.c_size_t(), ctypes.create_string_buffer(64), ctypes.c_uint64(), ctypes.c_uint8(), ctypes.c_int()
    st = L.h_tx_prepare(rlp, len(rlp), cid, len(cid), kind, pre, len(pre), ctypes.byref(n), rs, ctypes.byref(v),
                        ctypes.byref(vbig), ctypes.byref(hs))
    return st, pre.raw[:n.value], rs.raw, v.value, vbig.value


def vectors():
    g = golden("tx.json")
    return [(bytes.fromhex(v["rlp"]), 1, 0) for v in g["eip155_chain1"]] + \
           [(bytes.fromhex(v["rlp"]), 0, 1) for v in g["homestead"] + g["homestead_sighash"]]


def test_reference_vectors(txh, oracle):
    for rlp, cid, kind in vectors():
        st, pre, rs, v, vbig = prepare(txh, rlp, cid, kind)
        ost, sh = oracle.tx_sighash(rlp, cid, kind)
        assert st == ST_OK == ost and vbig == 0
        assert oracle.keccak256(pre) == sh
        # an EIP155 signer takes unprotected txs through the Homestead rules; a wrong chain id fails
        if kind == 0:
            assert prepare(txh, rlp, 2, 0)[0] == ST_INVALID_CHAIN_ID


def mutate(rng, b):
    b = bytearray(b)
    op = rng.randrange(6)
    if op == 0 and len(b) > 1:
        del b[rng.randrange(1, len(b)):]                    # truncate
    elif op == 1:
        i = rng.randrange(len(b))
        b[i] ^= 1 << rng.randrange(8)                        # bit flip
    elif op == 2:
        b.insert(rng.randrange(len(b) + 1), rng.randrange(256))  # insert
    elif op == 3:
        i = rng.randrange(min(len(b), 4))                    # a list / length prefix byte
        b[i] = rng.choice([0x80, 0x81, 0xb7, 0xb8, 0xb9, 0xbf, 0xc0, 0xf7, 0xf8, 0xf9, 0xff, b[i] ^ 0x08])
    elif op == 4:
        i = rng.randrange(len(b))
        b[i] = rng.choice([0x00, 0x80, 0x81, 0xa0, 0xa1, 0xc0, 0xff])  # an item prefix inside
    else:
        b += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 4)))  # trailing bytes
    return bytes(b)


def test_malformed_variants_agree_with_oracle(txh, oracle):
    """Decode-stage statuses equal the oracle's (BAD_RLP, INVALID_CHAIN_ID, INVALID_SIG from > 8-bit V
    or > 256-bit R/S); when the decoder accepts, the oracle must not reject at the decode stage and
    the preimage hashes to the oracle's sighash."""
    rng = random.Random(31)
    seen = {}
    for rlp, cid, kind in vectors():
        for _ in range(1500):
            m = mutate(rng, rlp)
            st, pre, rs, v, vbig = prepare(txh, m, cid, kind)
            ost, _ = oracle.tx_sender(m, cid, kind)
            seen[st] = seen.get(st, 0) + 1
            if st == ST_OK and vbig == 0:
                assert ost not in (ST_BAD_RLP, ST_INVALID_CHAIN_ID), (m.hex(), ost)
                hst, sh = oracle.tx_sighash(m, cid, kind)
                assert hst == 0 and oracle.keccak256(pre) == sh, m.hex()
            elif st == ST_OK:  # V or R/S too wide: the kernel reports ErrInvalidSig
                assert ost == ST_INVALID_SIG, (m.hex(), ost)
            else:
                assert st == ost, (m.hex(), st, ost)
    assert seen.get(ST_BAD_RLP, 0) > 1000 and seen.get(ST_OK, 0) > 100, seen
