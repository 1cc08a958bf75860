"""TEST INFRASTRUCTURE ONLY — ctypes loader for the CPU oracle and the reference build.

``liboracle.so`` is our plain-C restatement of the reference algorithms (gsv_oracle.c);
``_ref/libgsvref.so`` is the reference's own C code (libsecp256k1 with geth's cgo
defines + ethash sha3.c) compiled from /root/reference by ``make -C oracle ref``.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / CPU baseline. The product package (geth-sharding_amd/gsv) never
imports it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


def _ptr(a):
    return a.ctypes.data_as(c_u8p)


def build():
    subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


def lib():
    global _LIB
    if _LIB is None:
        # GSV_ORACLE_LIB: another build of the same sources (tools/sanitize.sh: ASan/UBSan)
        path = os.environ.get("GSV_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_keccak256.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_keccak_sponge.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int,
                                           ctypes.c_uint8, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_ecrecover.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_ecrecover_batch.argtypes = [c_u8p, c_u8p, ctypes.c_long, c_u8p, c_u8p, ctypes.c_int]
        L.oracle_tx_sender.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t,
                                       ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_tx_sighash.argtypes = L.oracle_tx_sender.argtypes
        L.oracle_recover_plain.argtypes = [ctypes.c_char_p, ctypes.c_char_p,
                                           ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_derive_sha_bytes.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_char_p]
        L.oracle_trie_root.argtypes = [c_u8p, c_u64p, c_u8p, c_u64p, ctypes.c_long, ctypes.c_char_p]
        L.oracle_secp_pubkey.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_secp_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_blob_serialize.argtypes = [c_u8p, c_u64p, c_u8p, ctypes.c_long, c_u8p, ctypes.c_long]
        L.oracle_blob_serialize.restype = ctypes.c_long
        L.oracle_blob_deserialize.argtypes = [c_u8p, ctypes.c_size_t, c_u8p, c_u64p, c_u8p, ctypes.c_long]
        L.oracle_blob_deserialize.restype = ctypes.c_long
        L.oracle_bn256_pairing_check.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_bn256_miller.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_bn256_final_exp.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_bn256_g1_mul.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_bn256_g2_mul.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        L.oracle_bn256_g2_check.argtypes = [ctypes.c_char_p]
        L.oracle_bn256_fp_mul_count.argtypes = [ctypes.c_int]
        L.oracle_bn256_fp_mul_count.restype = ctypes.c_uint64
        _LIB = L
    return _LIB


def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "libgsvref.so"))


def ref():
    """The reference's own C code (libsecp256k1 + ethash sha3), or None if not built."""
    global _REF
    if _REF is None and ref_available():
        R = ctypes.CDLL(os.path.join(HERE, "_ref", "libgsvref.so"))
        R.gsvref_ecrecover.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        R.gsvref_ecrecover_many.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_long]
        R.gsvref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        R.gsvref_pubkey.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        R.gsvref_keccak256.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        R.gsvref_keccak256_many.argtypes = [c_u8p, c_u8p, c_u64p, ctypes.c_long]
        R.gsvref_init()
        _REF = R
    return _REF


# ---------------------------------------------------------------- convenience wrappers
def keccak256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().oracle_keccak256(data, len(data), out)
    return out.raw


def sha3_256(data: bytes) -> bytes:
    """FIPS SHA3-256 through the same permutation (dsbyte 0x06), to pin Keccak-f."""
    out = ctypes.create_string_buffer(32)
    lib().oracle_keccak_sponge(data, len(data), 136, 0x06, out, 32)
    return out.raw


def ecrecover(msg32: bytes, sig65: bytes):
    """Returns (rc, pub65): rc 1 ok / 0 fail / -1 bad recid (ext.h + secp256.go semantics)."""
    pub = ctypes.create_string_buffer(65)
    rc = lib().oracle_ecrecover(pub, sig65, msg32)
    return rc, (pub.raw if rc == 1 else None)


def ecrecover_batch(msgs: np.ndarray, sigs: np.ndarray, threads: int = 8):
    n = msgs.shape[0]
    msgs = np.ascontiguousarray(msgs, dtype=np.uint8)
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8)
    pub = np.zeros((n, 65), np.uint8)
    st = np.zeros(n, np.uint8)
    lib().oracle_ecrecover_batch(_ptr(msgs), _ptr(sigs), n, _ptr(pub), _ptr(st), threads)
    return pub, st


def tx_sender(rlp: bytes, chain_id: int = 1, signer: int = 0):
    """signer: 0 EIP155Signer(chain_id), 1 HomesteadSigner, 2 FrontierSigner."""
    cid = chain_id.to_bytes((chain_id.bit_length() + 7) // 8, "big") if chain_id else b""
    out = ctypes.create_string_buffer(20)
    st = lib().oracle_tx_sender(out, rlp, len(rlp), cid, len(cid), signer)
    return st, (out.raw if st == 0 else None)


def tx_sighash(rlp: bytes, chain_id: int = 1, signer: int = 0):
    cid = chain_id.to_bytes((chain_id.bit_length() + 7) // 8, "big") if chain_id else b""
    out = ctypes.create_string_buffer(32)
    st = lib().oracle_tx_sighash(out, rlp, len(rlp), cid, len(cid), signer)
    return st, out.raw


def derive_sha_bytes(body) -> bytes:
    b = np.frombuffer(bytes(body), np.uint8) if not isinstance(body, np.ndarray) else body
    b = np.ascontiguousarray(b, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    lib().oracle_derive_sha_bytes(_ptr(b) if b.size else None, b.size, out)
    return out.raw


def trie_root(pairs) -> bytes:
    keys = b"".join(k for k, _ in pairs)
    vals = b"".join(v for _, v in pairs)
    koff = np.cumsum([0] + [len(k) for k, _ in pairs]).astype(np.uint64)
    voff = np.cumsum([0] + [len(v) for _, v in pairs]).astype(np.uint64)
    ka = np.frombuffer(keys + b"\0", np.uint8)
    va = np.frombuffer(vals + b"\0", np.uint8)
    out = ctypes.create_string_buffer(32)
    rc = lib().oracle_trie_root(_ptr(ka), koff.ctypes.data_as(c_u64p), _ptr(va),
                                voff.ctypes.data_as(c_u64p), len(pairs), out)
    assert rc == 0
    return out.raw


def rlp_uint(i: int) -> bytes:
    """rlp/encode.go:390 writeUint: 0 -> 0x80, < 128 -> the byte, else 0x80+len || big-endian."""
    if i == 0:
        return b"\x80"
    if i < 128:
        return bytes([i])
    b = i.to_bytes((i.bit_length() + 7) // 8, "big")
    return bytes([0x80 + len(b)]) + b


def rlp_string(b: bytes) -> bytes:
    """rlp/encode.go:71-89 encodeString"""
    b = bytes(b)
    if len(b) == 1 and b[0] < 0x80:
        return b
    if len(b) < 56:
        return bytes([0x80 + len(b)]) + b
    lb = len(b).to_bytes((len(b).bit_length() + 7) // 8, "big")
    return bytes([0xb7 + len(lb)]) + lb + b


def rlp_list(payload: bytes) -> bytes:
    if len(payload) < 56:
        return bytes([0xc0 + len(payload)]) + payload
    lb = len(payload).to_bytes((len(payload).bit_length() + 7) // 8, "big")
    return bytes([0xf7 + len(lb)]) + lb + payload


def derive_sha(items) -> bytes:
    """core/types/derive_sha.go:32-41: trie of (rlp(uint(j)), GetRlp(j)) -> root (restated trie)."""
    if len(items) == 0:
        return bytes.fromhex("56e81f171bcc55a6ff8345e692c0f86e5b48e01b996cadc001622fb5e363b421")
    return trie_root([(rlp_uint(j), bytes(v)) for j, v in enumerate(items)])


def calculate_poc(body: bytes, salt: bytes) -> bytes:
    """sharding/collation.go:124-136: chunk root of salt||b0||salt||b1||... (salt for an empty body)."""
    body, salt = bytes(body), bytes(salt)
    if len(body) == 0:
        salted = salt
    else:
        a = np.frombuffer(body, np.uint8)
        m = np.empty((len(body), len(salt) + 1), np.uint8)
        m[:, :len(salt)] = np.frombuffer(salt, np.uint8)
        m[:, len(salt)] = a
        salted = m.tobytes()
    return derive_sha_bytes(salted)


def _rlp_bigint(x) -> bytes:
    x = 0 if x is None else int(x)
    return b"\x80" if x == 0 else rlp_string(x.to_bytes((x.bit_length() + 7) // 8, "big"))


def collation_header_rlp(shard_id, chunk_root, period, proposer, sig) -> bytes:
    """rlp(collationHeaderData) (sharding/collation.go:35-43; nil pointers/slices -> 0x80,
    rlp/encode.go:545-581)."""
    f = [_rlp_bigint(shard_id),
         b"\x80" if chunk_root is None else rlp_string(chunk_root),
         _rlp_bigint(period),
         b"\x80" if proposer is None else rlp_string(proposer),
         rlp_string(sig or b"")]
    return rlp_list(b"".join(f))


def collation_header_hash(shard_id, chunk_root, period, proposer, sig) -> bytes:
    """CollationHeader.Hash (sharding/collation.go:66-71)."""
    return keccak256(collation_header_rlp(shard_id, chunk_root, period, proposer, sig))


def secp_pubkey(seckey: bytes) -> bytes:
    out = ctypes.create_string_buffer(65)
    assert lib().oracle_secp_pubkey(out, seckey) == 1
    return out.raw


def secp_sign(msg32: bytes, seckey: bytes, nonce32: bytes) -> bytes:
    out = ctypes.create_string_buffer(65)
    assert lib().oracle_secp_sign(out, msg32, seckey, nonce32) == 1
    return out.raw


def blob_serialize(blobs, skip_evm=None) -> bytes:
    data = np.frombuffer(b"".join(blobs) + b"\0", np.uint8)
    off = np.cumsum([0] + [len(b) for b in blobs]).astype(np.uint64)
    sk = np.array(skip_evm if skip_evm is not None else [0] * len(blobs), np.uint8)
    cap = sum(((len(b) + 30) // 31) * 32 for b in blobs) + 32
    out = np.zeros(cap, np.uint8)
    w = lib().oracle_blob_serialize(_ptr(data), off.ctypes.data_as(c_u64p),
                                    _ptr(sk) if sk.size else None, len(blobs), _ptr(out), cap)
    assert w >= 0
    return out[:w].tobytes()


def blob_deserialize(data: bytes):
    d = np.frombuffer(data + b"\0", np.uint8)
    nmax = len(data) // 32 + 1
    out = np.zeros(len(data) + 1, np.uint8)
    off = np.zeros(nmax + 1, np.uint64)
    sk = np.zeros(nmax, np.uint8)
    nb = lib().oracle_blob_deserialize(_ptr(d), len(data), _ptr(out), off.ctypes.data_as(c_u64p),
                                       _ptr(sk), nmax)
    assert nb >= 0
    return [(out[off[i]:off[i + 1]].tobytes(), int(sk[i])) for i in range(nb)]


def pairing_check(data: bytes):
    """1 true / 0 false / -1 bad input (core/vm/contracts.go:333-360 semantics)."""
    return lib().oracle_bn256_pairing_check(data, len(data))


def bn256_g1_mul(k: int, point64: bytes | None = None):
    """k * P in the precompile encoding (P = G1 generator when None); None on bad input."""
    out = ctypes.create_string_buffer(64)
    rc = lib().oracle_bn256_g1_mul(out, point64, (k % 2**256).to_bytes(32, "big"))
    return None if rc else out.raw


def bn256_g2_mul(k: int, point128: bytes | None = None):
    """k * Q in the precompile encoding (Q = G2 generator when None); None on bad input."""
    out = ctypes.create_string_buffer(128)
    rc = lib().oracle_bn256_g2_mul(out, point128, (k % 2**256).to_bytes(32, "big"))
    return None if rc else out.raw


def bn256_g2_check(point128: bytes) -> bool:
    return lib().oracle_bn256_g2_check(point128) == 0


def bn256_miller(pair192: bytes):
    out = ctypes.create_string_buffer(384)
    rc = lib().oracle_bn256_miller(pair192, out)
    return None if rc else out.raw


def bn256_fp_muls(inp: bytes):
    """F_p multiplications the reference algorithm spends on one precompile input."""
    L = lib()
    L.oracle_bn256_fp_mul_count(1)
    L.oracle_bn256_pairing_check(inp, len(inp))
    return int(L.oracle_bn256_fp_mul_count(1))
