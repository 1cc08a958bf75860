"""Mirror of the reference's crypto package entry points on the hot path, batched on the GPU.

    Keccak256(*data)            crypto/crypto.go:43-49
    Keccak256Hash(*data)        crypto/crypto.go:53-60
    Ecrecover(hash, sig)        crypto/signature_cgo.go:31-33 -> secp256k1.RecoverPubkey (secp256.go:105-122)
    SigToPub(hash, sig)         crypto/signature_cgo.go:36-44 (returns the 65-byte key here)
    EcrecoverBatch(...)         batch form used by the notary / tx pool hooks
    Keccak256Batch(msgs)        batch form
    Ecrecover precompile        core/vm/contracts.go:70-101 (EcrecoverPrecompile.Run / RunBatch)

Errors mirror crypto/secp256k1/secp256.go:54-62 and are raised as exceptions.
"""
from __future__ import annotations

import numpy as np

from . import _lib, default_context


class ErrInvalidMsgLen(ValueError):
    """invalid message length, need 32 bytes"""


class ErrInvalidSignatureLen(ValueError):
    """invalid signature length"""


class ErrInvalidRecoveryID(ValueError):
    """invalid signature recovery id"""


class ErrRecoverFailed(ValueError):
    """recovery failed"""


def Keccak256(*data) -> bytes:
    msg = b"".join(bytes(d) for d in data)
    return bytes(default_context().keccak256_batch([msg])[0])


Keccak256Hash = Keccak256


def Keccak256Batch(msgs, ctx=None) -> np.ndarray:
    return (ctx or default_context()).keccak256_batch(list(msgs))


def _check_lengths(msg: bytes, sig: bytes):
    # crypto/secp256k1/secp256.go:106-111 + checkSignature :171-178
    if len(msg) != 32:
        raise ErrInvalidMsgLen("invalid message length, need 32 bytes")
    if len(sig) != 65:
        raise ErrInvalidSignatureLen("invalid signature length")
    if sig[64] >= 4:
        raise ErrInvalidRecoveryID("invalid signature recovery id")


def Ecrecover(hash: bytes, sig: bytes) -> bytes:
    """Returns the uncompressed public key (65 bytes) that created the signature."""
    hash, sig = bytes(hash), bytes(sig)
    _check_lengths(hash, sig)
    pub, _, st = default_context().ecrecover_batch(np.frombuffer(hash, np.uint8)[None],
                                                   np.frombuffer(sig, np.uint8)[None])
    if st[0] != _lib.ST_OK:
        raise ErrRecoverFailed("recovery failed")
    return bytes(pub[0])


SigToPub = Ecrecover


def EcrecoverBatch(hashes, sigs, want_pub=True, want_addr=False, ctx=None):
    """Batch ecrecover: per-item status codes (GSV_ST_*) instead of exceptions."""
    return (ctx or default_context()).ecrecover_batch(hashes, sigs, want_pub=want_pub,
                                                      want_addr=want_addr)


def PubkeyToAddress(pub65: bytes) -> bytes:
    """crypto/crypto.go:194-197: Keccak256(pub[1:])[12:]."""
    return Keccak256(bytes(pub65)[1:])[12:]


def ValidateSignatureValues(v: int, r: int, s: int, homestead: bool) -> bool:
    """crypto/crypto.go:181-192 (host-side predicate; the kernels apply the same rule per lane)."""
    n = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    if r < 1 or s < 1:
        return False
    if homestead and s > n // 2:
        return False
    return r < n and s < n and v in (0, 1)


class EcrecoverPrecompile:
    """PrecompiledContract{RequiredGas, Run} for address 0x01 (core/vm/contracts.go:70-101)."""

    ECRECOVER_GAS = 3000  # params.EcrecoverGas

    def RequiredGas(self, input: bytes) -> int:
        return self.ECRECOVER_GAS

    def Run(self, input: bytes, ctx=None):
        """32-byte left-padded signer address, or None where the reference returns (nil, nil)."""
        out, ok = self.RunBatch([bytes(input)], ctx)
        return bytes(out[0]) if ok[0] else None

    def RunBatch(self, inputs, ctx=None):
        return (ctx or default_context()).ecrecover_precompile_batch(list(inputs))
