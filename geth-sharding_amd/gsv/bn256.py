"""Mirror of the reference's BN254 pairing entry points, batched on the GPU.

    PairingCheck(a, b)          crypto/bn256/bn256_fast.go -> cloudflare/bn256.go:313-327
    PairingCheckBatch(inputs)   the batch form: one verdict per precompile input
    Bn256Pairing.Run(input)     core/vm/contracts.go:333-360 (true32Byte / false32Byte / error)

Points use the precompile encoding: G1 = x || y, G2 = x.imag || x.real || y.imag || y.real,
32-byte big-endian words (bn256.go:120-164, :256-306).  Malformed points raise
ErrMalformedPoint where the reference's Unmarshal returns an error.
"""
from __future__ import annotations

import numpy as np

from . import _lib, default_context


class ErrBadPairingInput(ValueError):
    """bad elliptic curve pairing size (core/vm/contracts.go:315, errBadPairingInput)"""


class ErrMalformedPoint(ValueError):
    """bn256: coordinate exceeds modulus / malformed point (cloudflare/bn256.go)"""


TRUE32 = bytes(31) + b"\x01"
FALSE32 = bytes(32)


def PairingCheckBatch(inputs, ctx=None) -> np.ndarray:
    return (ctx or default_context()).pairing_check_batch(list(inputs))


def PairingCheck(a, b, ctx=None) -> bool:
    """a: list of 64-byte G1 encodings, b: list of 128-byte G2 encodings."""
    if len(a) != len(b):
        raise ValueError("PairingCheck: len(a) != len(b)")
    inp = b"".join(bytes(x) + bytes(y) for x, y in zip(a, b))
    v = PairingCheckBatch([inp], ctx)[0]
    if v == _lib.PAIRING_BAD_INPUT:
        raise ErrMalformedPoint("bn256: malformed point")
    return bool(v == _lib.PAIRING_TRUE)


class Bn256Pairing:
    """PrecompiledContract{RequiredGas, Run} for address 0x08 (core/vm/contracts.go:325-360)."""

    PAIRING_BASE_GAS = 100000   # params.Bn256PairingBaseGas
    PAIRING_PER_POINT_GAS = 80000  # params.Bn256PairingPerPointGas

    def RequiredGas(self, input: bytes) -> int:
        return self.PAIRING_BASE_GAS + (len(input) // 192) * self.PAIRING_PER_POINT_GAS

    def Run(self, input: bytes, ctx=None) -> bytes:
        if len(input) % 192:
            raise ErrBadPairingInput("bad elliptic curve pairing size")
        v = PairingCheckBatch([bytes(input)], ctx)[0]
        if v == _lib.PAIRING_BAD_INPUT:  # newCurvePoint / newTwistPoint error (contracts.go:344-351)
            raise ErrMalformedPoint("bn256: malformed point")
        return TRUE32 if v == _lib.PAIRING_TRUE else FALSE32
