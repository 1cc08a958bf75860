"""Mirror of the reference's collation validation entry points (package sharding + types.DeriveSha),
batched on the GPU.

    DeriveSha(list)                  core/types/derive_sha.go:32-41 (any DerivableList: list of GetRlp(j))
    DeriveShaBatch(lists)            batch form: tx roots (core/block_validator.go:70), receipt roots (:92)
    CollationHeader.Hash()           sharding/collation.go:66-71
    Collation.CalculateChunkRoot()   sharding/collation.go:115-119
    Collation.CalculatePOC(salt)     sharding/collation.go:124-136
    VerifyProposerSignatures(hdrs)   proposer signature over the unsigned header hash, as made by
                                     SMCClient.Sign (sharding/mainchain/smc_client.go:245-248) at
                                     sharding/proposer/proposer.go:83 (the reference never checks it)

Integers (ShardID, Period) are Python ints (the reference's *big.Int); None stands for a nil pointer.
"""
from __future__ import annotations

import numpy as np

from . import _lib, default_context

COLLATION_SIZE_LIMIT = 1 << 20  # sharding/collation.go:45


class ErrProposerMismatch(ValueError):
    """recovered proposer signature address differs from the header's ProposerAddress"""


def DeriveSha(items, ctx=None) -> bytes:
    """types.DeriveSha over a list whose GetRlp(j) is items[j] (bytes)."""
    return bytes((ctx or default_context()).derive_sha_batch([list(items)])[0])


def DeriveShaBatch(lists, ctx=None) -> np.ndarray:
    return (ctx or default_context()).derive_sha_batch([list(x) for x in lists])


def _int32(x) -> bytes:
    x = 0 if x is None else int(x)
    if x < 0:
        raise ValueError("rlp: cannot encode negative *big.Int")
    return x.to_bytes(32, "big")


def _pack_headers(headers):
    n = len(headers)
    sid = np.zeros((n, 32), np.uint8)
    root = np.zeros((n, 32), np.uint8)
    per = np.zeros((n, 32), np.uint8)
    prop = np.zeros((n, 20), np.uint8)
    sig = np.zeros((n, 65), np.uint8)
    nil = np.zeros(n, np.uint8)
    for i, h in enumerate(headers):
        sid[i] = np.frombuffer(_int32(h.ShardID()), np.uint8)
        per[i] = np.frombuffer(_int32(h.Period()), np.uint8)
        if h.ChunkRoot() is None:
            nil[i] |= 1
        else:
            root[i] = np.frombuffer(bytes(h.ChunkRoot()), np.uint8)
        if h.ProposerAddress() is None:
            nil[i] |= 2
        else:
            prop[i] = np.frombuffer(bytes(h.ProposerAddress()), np.uint8)
        s = h.Sig()
        if not s:
            nil[i] |= 4
        elif len(s) != 65:
            raise ValueError("proposer signature must be 65 bytes [R || S || V]")
        else:
            sig[i] = np.frombuffer(bytes(s), np.uint8)
    return sid, root, per, prop, sig, nil


class CollationHeader:
    """sharding/collation.go:29-43 (collationHeaderData fields behind getters)."""

    def __init__(self, shard_id, chunk_root, period, proposer_address, proposer_signature=None):
        self._shard_id = shard_id
        self._chunk_root = None if chunk_root is None else bytes(chunk_root)
        self._period = period
        self._proposer = None if proposer_address is None else bytes(proposer_address)
        self._sig = None if proposer_signature is None else bytes(proposer_signature)

    def ShardID(self):
        return self._shard_id

    def Period(self):
        return self._period

    def ChunkRoot(self):
        return self._chunk_root

    def ProposerAddress(self):
        return self._proposer

    def Sig(self):
        return self._sig

    def AddSig(self, sig: bytes):
        self._sig = bytes(sig)

    def Hash(self, ctx=None) -> bytes:
        return bytes(HeaderHashBatch([self], ctx)[0])


def HeaderHashBatch(headers, ctx=None) -> np.ndarray:
    """CollationHeader.Hash() for each header (signature included as set)."""
    h, _, _ = (ctx or default_context()).collation_header_verify_batch(*_pack_headers(headers))
    return h


def VerifyProposerSignatures(headers, ctx=None):
    """-> (signers (n,20), status (n,)): GSV_ST_OK when the signature over the unsigned header hash
    recovers ProposerAddress, GSV_ST_PROPOSER_MISMATCH when it recovers another address, else the
    recovery status (crypto.Ecrecover errors)."""
    _, signer, st = (ctx or default_context()).collation_header_verify_batch(*_pack_headers(headers))
    return signer, st


class Collation:
    """sharding/collation.go:15-27: header + serialized body."""

    def __init__(self, header: CollationHeader, body: bytes, transactions=None):
        self.header = header
        self.body = bytes(body)
        self.transactions = transactions

    def Header(self):
        return self.header

    def Body(self):
        return self.body

    def CalculateChunkRoot(self, ctx=None):
        root = bytes((ctx or default_context()).chunk_root_batch([self.body])[0])
        self.header._chunk_root = root

    def CalculatePOC(self, salt: bytes, ctx=None) -> bytes:
        return bytes((ctx or default_context()).collation_poc_batch([self.body], bytes(salt))[0])


def CalculatePOCBatch(bodies, salt: bytes, ctx=None) -> np.ndarray:
    return (ctx or default_context()).collation_poc_batch(list(bodies), bytes(salt))


__all__ = ["DeriveSha", "DeriveShaBatch", "CollationHeader", "Collation", "HeaderHashBatch",
           "VerifyProposerSignatures", "CalculatePOCBatch", "ErrProposerMismatch", "COLLATION_SIZE_LIMIT",
           "_lib"]
