"""Host build of the device secp256k1 field/group arithmetic (geth-sharding_amd/csrc/
secp256k1_fe9.cuh, 9 x 29-bit limbs with lazy reduction) checked against Python integers.

The header compiles as plain C++ for the host, so its magnitude bookkeeping — the claim that no
limb or 64-bit column ever overflows under the documented preconditions — is exercised here at
the extreme limb values each precondition admits, not only on random data.  CPU-only."""
import ctypes
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
P = 2**256 - 2**32 - 977
B = 7
M29 = 2**29 - 1
U9 = ctypes.c_uint32 * 9


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    from conftest import build_native
    return build_native("fe9_host.cpp", tmp_path_factory.mktemp("fe9") / "fe9_host.so")


def val(l):
    return sum(int(x) << (29 * i) for i, x in enumerate(l))


def rnd_limbs(rng, mag, top=None):
    """limbs < mag * 2^29 (limb 8 < top), half the time pinned at the bound."""
    hi = int(mag * 2**29)
    t = hi if top is None else top
    out = []
    for i in range(9):
        b = t if i == 8 else hi
        out.append(b - 1 if rng.random() < 0.3 else rng.randrange(b))
    return out


def from_int(x):
    return [(x >> (29 * i)) & M29 for i in range(9)]


def arr(l):
    return U9(*l)


def check_mag1(l):
    assert all(l[i] < 2**29 for i in (0, 1, 3, 4, 5, 6, 7)), l
    assert l[2] < 2**29 + 2**24 and l[8] < 2**24, l


MAG_PAIRS = [(1.04, 1.04), (1.04, 6.7), (6.7, 1.04), (2.08, 3.36), (3.36, 2.08), (2.64, 2.64), (1.04, 4.16), (4.16, 1.04)]


def test_mul_bounds_and_values(lib):
    rng = random.Random(11)
    r = U9()
    for ma, mb in MAG_PAIRS:
        assert ma * mb <= 7.0
        for _ in range(400):
            a, b = rnd_limbs(rng, ma), rnd_limbs(rng, mb)
            lib.h_mul(r, arr(a), arr(b))
            check_mag1(list(r))
            assert val(r) % P == val(a) * val(b) % P
            assert val(r) < 2**256 + 2**88


def test_sqr_bounds_and_values(lib):
    rng = random.Random(12)
    r = U9()
    for m in (1.04, 2, 2.64):
        for _ in range(600):
            a = rnd_limbs(rng, m)
            lib.h_sqr(r, arr(a))
            check_mag1(list(r))
            assert val(r) % P == val(a) ** 2 % P


def test_sub_neg_add(lib):
    rng = random.Random(13)
    r = U9()
    for M in range(1, 7):
        for ma in (1.04, 2, 3):
            if ma + M + 1 >= 8:
                continue
            for _ in range(200):
                a, b = rnd_limbs(rng, ma), rnd_limbs(rng, M)
                lib.h_sub(r, arr(a), arr(b), M)
                assert all(x < (ma + M + 1) * 2**29 for x in r)
                assert (val(r) - val(a) + val(b)) % P == 0


def test_normalize(lib):
    rng = random.Random(14)
    edge = [0, 1, P - 1, P, P + 1, 2**256 - 1, 2**256, 2**256 + 2**40, 2 * P - 1, 2**32 + 976, 2**32 + 977]
    cases = [from_int(x) for x in edge if x < 2**261] + [rnd_limbs(rng, 7.9) for _ in range(3000)]
    # values >= 2^256 with limb 2 at the weak bound, limbs at the magnitude ceiling
    cases += [[M29, M29, 2**29, M29, M29, M29, M29, M29, 2**24 - 1], [int(7.9 * 2**29)] * 9]
    for l in cases:
        w = arr(l)
        lib.h_norm_weak(w)
        check_mag1(list(w))
        assert val(w) % P == val(l) % P
        f = arr(l)
        lib.h_norm_full(f)
        assert val(f) == val(l) % P
        assert all(x <= M29 for x in f)
        # the cheap zero test on weakly normalised values agrees with the full one
        assert lib.h_is_zero_weak(w) == (val(l) % P == 0)


def test_is_zero_weak_edges(lib):
    """fe9_is_zero_weak on every weak form of 0 and p it can meet (normalize_weak outputs of
    multiples of p, and mul/sqr outputs with limb 2 up to 2^29 + 2^24) and on near misses."""
    rng = random.Random(15)
    vals = [0, P, 2 * P, 3 * P, 7 * P, 1, P - 1, P + 1, 2**256, 2**29, 2**58]
    for x in vals:
        l = from_int(x) if x < 2**261 else None
        w = arr(l)
        lib.h_norm_weak(w)
        assert lib.h_is_zero_weak(w) == (x % P == 0)
    for _ in range(2000):  # product outputs: limb 2 in [0, 2^29 + 2^24), others canonical
        l = [rng.randrange(2**29) for _ in range(9)]
        l[2] = rng.randrange(2**29 + 2**24)
        l[8] = rng.randrange(2**24)
        if rng.random() < 0.3:
            l = list(from_int(P if rng.random() < 0.5 else 0))
        assert lib.h_is_zero_weak(arr(l)) == (val(l) % P == 0)


def test_words_roundtrip(lib):
    rng = random.Random(15)
    W8 = ctypes.c_uint32 * 8
    for _ in range(300):
        x = rng.randrange(P)
        w = W8(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
        l = U9()
        lib.h_from_words(l, w)
        assert list(l) == from_int(x)
        w2 = W8()
        lib.h_to_words(w2, l)
        assert list(w2) == list(w)


def test_inv_sqrt(lib):
    rng = random.Random(16)
    r = U9()
    for _ in range(20):
        x = rng.randrange(1, P)
        lib.h_inv(r, arr(rnd_limbs_val(rng, x)))
        assert val(r) * x % P == 1
        s = x * x % P
        ok = lib.h_sqrt(r, arr(from_int(s)))
        assert ok == 1 and (val(r) ** 2 - s) % P == 0
        # a non-residue: -s is one (p = 3 mod 4) unless s == 0
        ok = lib.h_sqrt(r, arr(from_int((-s) % P)))
        assert ok == 0


def test_pow_pm3_4(lib):
    """fe9_pow_pm3_4 (the recovery's one exponentiation, recover_dev.cuh recover_tail_twisted):
    a^((p-3)/4), i.e. 1/sqrt(a) for a square a, on redundant inputs"""
    rng = random.Random(17)
    r = U9()
    for _ in range(20):
        x = rng.randrange(1, P)
        lib.h_pow_pm3_4(r, arr(rnd_limbs_val(rng, x)))
        assert val(r) % P == pow(x, (P - 3) // 4, P)
        s = x * x % P
        lib.h_pow_pm3_4(r, arr(from_int(s)))
        w = val(r) % P
        assert (w * w * s) % P == 1  # 1 / sqrt(s)^2 * s


def rnd_limbs_val(rng, x):
    """a magnitude-2 representation of x: x + k p split with limbs up to 2^30"""
    l = from_int(x)
    # add p limb-wise with a random subset shifted into a redundant form
    for i in range(8):
        if rng.random() < 0.5 and l[i + 1] > 0:
            l[i] += 2**29
            l[i + 1] -= 1
    assert val(l) == x
    return l


# ---------------------------------------------------------------- group ops vs affine Python
def inv(x):
    return pow(x, P - 2, P)


def aff_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    (x1, y1), (x2, y2) = p1, p2
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * inv(2 * y1) % P
    else:
        lam = (y2 - y1) * inv(x2 - x1) % P
    x3 = (lam * lam - x1 - x2) % P
    return x3, (lam * (x1 - x3) - y1) % P


GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def mul_pt(k, pt):
    acc = None
    for bit in bin(k)[2:]:
        acc = aff_add(acc, acc)
        if bit == "1":
            acc = aff_add(acc, pt)
    return acc


def to_jac(rng, pt):
    z = rng.randrange(1, P)
    x, y = pt
    X, Y = x * z * z % P, y * z * z * z % P
    # X, Y magnitude 1; Z magnitude 2 (redundant form)
    return from_int(X) + from_int(Y) + rnd_limbs_val(rng, z)


def from_jac(l):
    X, Y, Z = val(l[0:9]) % P, val(l[9:18]) % P, val(l[18:27]) % P
    zi = inv(Z)
    return X * zi * zi % P, Y * zi * zi * zi % P


def test_dbl_add(lib):
    rng = random.Random(17)
    U27, U18 = ctypes.c_uint32 * 27, ctypes.c_uint32 * 18
    for _ in range(25):
        p1 = mul_pt(rng.randrange(1, 2**64), (GX, GY))
        p2 = mul_pt(rng.randrange(1, 2**64), (GX, GY))
        jp = U27(*to_jac(rng, p1))
        out = U27()
        lib.h_dbl(out, jp)
        o = list(out)
        check_mag1(o[0:9]), check_mag1(o[9:18])
        assert all(x < 2 * 2**29 for x in o[18:27])
        assert from_jac(o) == aff_add(p1, p1)
        # mixed add with q.y negated at magnitude 2 half the time
        x2, y2 = p2
        ql = from_int(x2) + (from_int(y2) if rng.random() < 0.5 else rnd_limbs_val(rng, y2))
        h, rr = U9(), U9()
        lib.h_add_ge(out, h, rr, jp, U18(*ql))
        o = list(out)
        check_mag1(o[0:9]), check_mag1(o[9:18])
        assert all(x < 2 * 2**29 for x in o[18:27])
        assert from_jac(o) == aff_add(p1, p2)


def test_add_ge_exceptional_and_general_add(lib):
    rng = random.Random(18)
    U27, U18 = ctypes.c_uint32 * 27, ctypes.c_uint32 * 18
    out = U27()
    for _ in range(12):
        p1 = mul_pt(rng.randrange(1, 2**64), (GX, GY))
        p2 = mul_pt(rng.randrange(1, 2**64), (GX, GY))
        jp = U27(*to_jac(rng, p1))
        for q, want in ((p2, aff_add(p1, p2)), (p1, aff_add(p1, p1)), ((p1[0], P - p1[1]), None)):
            ql = U18(*(from_int(q[0]) + rnd_limbs_val(rng, q[1])))
            inf = lib.h_add_ge_full(out, jp, 0, ql)
            if want is None:
                assert inf == 1
            else:
                assert inf == 0 and from_jac(list(out)) == want
        # p = infinity -> q
        ql = U18(*(from_int(p2[0]) + rnd_limbs_val(rng, p2[1])))
        assert lib.h_add_ge_full(out, jp, 1, ql) == 0 and from_jac(list(out)) == p2
        # general add: generic, doubling, inverse, infinities
        jq = U27(*to_jac(rng, p2))
        assert lib.h_add(out, jp, 0, jq, 0) == 0 and from_jac(list(out)) == aff_add(p1, p2)
        jp2 = U27(*to_jac(rng, p1))
        assert lib.h_add(out, jp, 0, jp2, 0) == 0 and from_jac(list(out)) == aff_add(p1, p1)
        jn = U27(*to_jac(rng, (p1[0], P - p1[1])))
        assert lib.h_add(out, jp, 0, jn, 0) == 1
        assert lib.h_add(out, jp, 1, jq, 0) == 0 and from_jac(list(out)) == p2
        assert lib.h_add(out, jp, 0, jq, 1) == 0 and from_jac(list(out)) == p1


def test_build_r_table(lib):
    """T[e] are (2e+1) R on the isomorphic curve: with zfac, (T.x zfac^-2... ) -> check through
    the relation that the Jacobian point (T.x, T.y, zfac) on E is (2e+1) R."""
    rng = random.Random(19)
    U72 = ctypes.c_uint32 * 72
    for _ in range(8):
        R = mul_pt(rng.randrange(1, 2**64), (GX, GY))
        T, z = U72(), U9()
        lib.h_build_table(T, z, arr(from_int(R[0])), arr(from_int(R[1])))
        zf = val(z) % P
        for e in range(4):
            tx, ty = val(T[18 * e:18 * e + 9]) % P, val(T[18 * e + 9:18 * e + 18]) % P
            zi = inv(zf)
            assert (tx * zi * zi % P, ty * zi * zi * zi % P) == mul_pt(2 * e + 1, R)


N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
BN_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583


@pytest.fixture(scope="module", params=[0, 1], ids=["const-time", "var-time"])
def inv_lib(request, tmp_path_factory):
    """the host harness built with each divstep form (modinv30.cuh MI30_VAR)"""
    from conftest import build_native
    return build_native("fe9_host.cpp", tmp_path_factory.mktemp("fe9v") / f"fe9_host_v{request.param}.so",
                        defines=[f"MI30_VAR={request.param}"])


def test_safegcd_modinv(inv_lib):
    """modinv30.cuh (Bernstein-Yang divsteps, constant- and variable-time) against pow(x, -1, m) for
    m = n, p and the BN254 prime."""
    lib = inv_lib
    rng = random.Random(20)
    W8 = ctypes.c_uint32 * 8
    for which, m in ((0, N_ORDER), (1, P), (2, BN_P)):
        xs = [0, 1, 2, 3, m - 1, m - 2, (m - 1) // 2, 2**255, 2**128 + 1, 0xFFFFFFFF] + [rng.randrange(1, m) for _ in range(3000)]
        xs += [rng.getrandbits(rng.randrange(1, 256)) % m for _ in range(500)]
        for x in xs:
            out = W8()
            lib.h_modinv(out, W8(*[(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]), which)
            got = sum(v << (32 * i) for i, v in enumerate(out))
            assert got == (pow(x, -1, m) if x else 0), (which, hex(x), hex(got))
