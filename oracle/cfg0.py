"""TEST INFRASTRUCTURE ONLY — the configs[0] workload and its CPU path.

configs[0] (BASELINE.json): "core/types Sender recovery of 10k synthetic EIP-155 signed txs via
crypto.Ecrecover (libsecp256k1 cgo) on CPU".  The txs follow SURVEY.md §8d Cfg1: key_i = 1 +
(Keccak256("gsv-key" || le64(i)) mod (n - 1)), nonce = i mod 128, gasPrice 20 Gwei, gas 21,000,
to = Keccak256("gsv-to" || le64(i))[12:], value = i, no data, chainId 1, signed with RFC6979 by the
reference's libsecp256k1 (oracle/_ref) — or by the oracle signer with a Keccak-derived nonce where
the reference build is absent.

The CPU path is types.Sender (core/types/transaction_signing.go:72-89,127-165): RLP decode, sighash
RLP, Keccak, recovery, address Keccak — the RLP layer from the oracle's restatement (Go cannot run
here), the crypto from the reference's own C when oracle/_ref is built (use_reference_crypto).
Only tests/ and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import struct
import time

import numpy as np

from . import oracle as O

N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
CHAIN_ID = 1


def _rlp_int(x: int) -> bytes:
    return b"\x80" if x == 0 else O.rlp_string(x.to_bytes((x.bit_length() + 7) // 8, "big"))


def eip155_txs(n: int):
    """-> (list of signed tx RLP, expected sender addresses (n, 20) uint8)"""
    R = O.ref()
    txs, addrs = [], np.zeros((n, 20), np.uint8)
    for i in range(n):
        k = 1 + int.from_bytes(O.keccak256(b"gsv-key" + struct.pack("<Q", i)), "big") % (N_ORDER - 1)
        key = k.to_bytes(32, "big")
        to = O.keccak256(b"gsv-to" + struct.pack("<Q", i))[12:]
        fields = [_rlp_int(i % 128), _rlp_int(20 * 10**9), _rlp_int(21000), O.rlp_string(to), _rlp_int(i),
                  O.rlp_string(b"")]
        sighash = O.keccak256(O.rlp_list(b"".join(fields + [_rlp_int(CHAIN_ID), _rlp_int(0), _rlp_int(0)])))
        if R is not None:
            sig = ctypes.create_string_buffer(65)
            assert R.gsvref_sign(sig, sighash, key) == 1
            sig = sig.raw
        else:
            nonce = (1 + int.from_bytes(O.keccak256(b"gsv-nonce" + struct.pack("<Q", i)), "big") % (N_ORDER - 1))
            sig = O.secp_sign(sighash, key, nonce.to_bytes(32, "big"))
        r, s, recid = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:64], "big"), sig[64]
        v = recid + 35 + 2 * CHAIN_ID
        txs.append(O.rlp_list(b"".join(fields + [_rlp_int(v), _rlp_int(r), _rlp_int(s)])))
        addrs[i] = np.frombuffer(O.keccak256(O.secp_pubkey(key)[1:])[12:], np.uint8)
    return txs, addrs


def use_reference_crypto() -> str:
    """Route the oracle's Sender through the reference's Keccak + libsecp256k1 (oracle/_ref).
    Returns the cpu_baseline kind: "reference" or "port" (restatement only)."""
    L = O.lib()
    L.oracle_set_crypto.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    R = O.ref()
    if R is None:
        L.oracle_set_crypto(None, None)
        return "port"
    R.gsvref_init()
    L.oracle_set_crypto(ctypes.cast(R.gsvref_keccak256, ctypes.c_void_p), ctypes.cast(R.gsvref_ecrecover,
                                                                                     ctypes.c_void_p))
    return "reference"


def sender_many(flat: np.ndarray, off: np.ndarray, n: int, threads: int, chain_id: int = CHAIN_ID):
    """types.Sender with EIP155Signer(chain_id) over n txs on `threads` C threads -> (addr, status, seconds)"""
    L = O.lib()
    u8 = ctypes.POINTER(ctypes.c_uint8)
    L.oracle_tx_sender_many.argtypes = [u8, ctypes.POINTER(ctypes.c_uint64), ctypes.c_long, ctypes.c_char_p,
                                        ctypes.c_size_t, ctypes.c_int, u8, u8, ctypes.c_int]
    cid = chain_id.to_bytes((chain_id.bit_length() + 7) // 8, "big") if chain_id else b""
    addr = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    t0 = time.perf_counter()
    L.oracle_tx_sender_many(flat.ctypes.data_as(u8), off.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), n, cid,
                            len(cid), 0, addr.ctypes.data_as(u8), st.ctypes.data_as(u8), threads)
    return addr, st, time.perf_counter() - t0
