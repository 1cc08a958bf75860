"""CPU check of the digest permutation's last round (geth-sharding_amd/csrc/keccak_dev.cuh
keccakf_split_digest): after 23 full rounds, the last round computes only state words 0..3 from theta's
five column parities, the diagonal A[6k] (x = y) through theta / rho / pi, and chi of row 0.  Restated
here with the kernel's own index formulas and compared with the full Keccak-f[1600]
(crypto/sha3/keccakf.go:39) on random states and on the oracle's Keccak-256 digests."""
import random

M64 = (1 << 64) - 1
RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
      0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
      0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
      0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
      0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
RHO = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]


def rot(v, r):
    return ((v << r) | (v >> (64 - r))) & M64 if r else v


def round_full(a, rc):
    c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
    d = [rot(c[(x + 1) % 5], 1) for x in range(5)]
    b = [0] * 25
    for i in range(25):
        x, y = i % 5, i // 5
        b[y + 5 * ((2 * x + 3 * y) % 5)] = rot(a[i] ^ c[(x + 4) % 5] ^ d[x], RHO[i])
    out = [b[(i // 5) * 5 + i % 5] ^ (~b[(i // 5) * 5 + (i % 5 + 1) % 5] & M64 & b[(i // 5) * 5 + (i % 5 + 2) % 5])
           for i in range(25)]
    out[0] ^= rc
    return out


def round_digest(a, rc):
    """The kernel's last round: B[k] = rot(theta(A)[6k], RHO[6k]) for k < 5, chi of words 0..3."""
    c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
    d = [rot(c[(x + 1) % 5], 1) for x in range(5)]
    b = [rot(a[6 * k] ^ c[(k + 4) % 5] ^ d[k], RHO[6 * k]) for k in range(5)]
    out = [b[x] ^ (~b[(x + 1) % 5] & M64 & b[(x + 2) % 5]) for x in range(4)]
    out[0] ^= rc
    return out


def keccakf(a, digest=False):
    for r in range(23):
        a = round_full(a, RC[r])
    return round_digest(a, RC[23]) if digest else round_full(a, RC[23])


def test_pi_places_the_diagonal_in_row_0():
    # pi: A[x + 5y] -> B[y + 5((2x + 3y) mod 5)]; row 0 of B is exactly the diagonal x = y, in order
    row0 = {y + 5 * ((2 * x + 3 * y) % 5): x + 5 * y for x in range(5) for y in range(5)
            if (2 * x + 3 * y) % 5 == 0}
    assert row0 == {k: 6 * k for k in range(5)}


def test_digest_round_matches_full_permutation_on_random_states():
    rng = random.Random(20261019)
    for _ in range(200):
        a = [rng.getrandbits(64) for _ in range(25)]
        assert keccakf(a, digest=True) == keccakf(a)[:4]


def test_digest_round_keccak256_vs_oracle(oracle):
    rng = random.Random(7)
    for n in (0, 1, 31, 32, 83, 135, 136, 137, 271, 272, 532, 1000):
        msg = bytes(rng.getrandbits(8) for _ in range(n))
        p = bytearray(msg) + b"\x01" + bytes((-(n + 1)) % 136)
        p[-1] |= 0x80
        a = [0] * 25
        for blk in range(len(p) // 136):
            for k in range(17):
                a[k] ^= int.from_bytes(p[136 * blk + 8 * k:136 * blk + 8 * k + 8], "little")
            last = blk == len(p) // 136 - 1
            a = keccakf(a, digest=last)
        digest = b"".join(w.to_bytes(8, "little") for w in a[:4])
        assert digest == oracle.keccak256(msg), n

