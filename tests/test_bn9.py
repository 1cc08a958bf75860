"""Host build of the BN254 9 x 29-bit Montgomery field and its F_p^2 / F_p^6 towers
(geth-sharding_amd/csrc/bn254_fe9.cuh, compiled as plain C++ through tests/native/bn9_host.cpp)
checked against Python integers.  CPU-only.

Every result is held to the magnitude its compile-time type claims — fqm<L, V>: limbs <= L (2^29 - 1) and
value < V p — at the extreme operands each precondition admits, not only on random data; the tower
products are checked against a Python restatement of the reference's tower (crypto/bn256/cloudflare
gfp2.go, gfp6.go: i^2 = -1, tau^3 = xi = i + 9), the Frobenius maps against a^p computed by
exponentiation (which checks the converted constants of tools/gen_bn9_consts.py independently)."""
import ctypes
import os
import random
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 2**261
RINV = pow(R, -1, P)
U9 = ctypes.c_uint32 * 9
I2 = ctypes.c_int * 2


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    from conftest import build_native
    global VS
    L = build_native("bn9_host.cpp", tmp_path_factory.mktemp("bn9") / "bn9_host.so")
    VS = L.h_vs()
    return L


def val(l):
    return sum(int(x) << (29 * i) for i, x in enumerate(l))


def limbs(x):
    return [(x >> (29 * i)) & (2**29 - 1) for i in range(8)] + [x >> 232]


def rnd(rng, L, V):
    """limbs <= L (2^29 - 1) and value < V p, limbs pinned at their bound a third of the time"""
    hi = L * (2**29 - 1)
    low = [hi if rng.random() < 0.35 else rng.randrange(hi + 1) for _ in range(8)]
    lv = sum(x << (29 * i) for i, x in enumerate(low))
    top = min(hi, (V * P - 1 - lv) >> 232)
    assert top >= 0
    t8 = top if rng.random() < 0.35 else rng.randrange(top + 1)
    return low + [t8]


def check(r, lv):
    L, V = lv
    assert all(x <= L * (2**29 - 1) for x in r), (list(r), L)
    assert val(r) < V * P, (val(r) / P, V)


def parse(name, n):
    return [int(x) for x in name.split("_")[-n:]]


MULS = ["h_mul_1_1_1_1", "h_mul_1_32_1_32", "h_mul_2_48_3_48", "h_mul_6_8_1_160", "h_mul_3_64_2_36", "h_mul_8_4_8_4"]
MUL2S = ["h_mul2_1_32_1_32_1_32_2_34", "h_mul2_2_40_1_32_2_40_2_36", "h_mul2_1_3_3_3_1_3_3_3"]
ADDSUBS = ["1_32_1_32", "3_40_5_48", "7_100_6_60", "2_160_1_160"]


def test_mul_bounds_and_values(lib):
    rng = random.Random(21)
    r, lv = U9(), I2()
    for nm in MULS:
        La, Va, Lb, Vb = parse(nm, 4)
        fn = getattr(lib, nm)
        for _ in range(300):
            a, b = rnd(rng, La, Va), rnd(rng, Lb, Vb)
            fn(r, lv, U9(*a), U9(*b))
            check(r, lv)
            assert val(r) % P == val(a) * val(b) * RINV % P


def test_mul2_bounds_and_values(lib):
    rng = random.Random(22)
    r, lv = U9(), I2()
    for nm in MUL2S:
        q = parse(nm, 8)
        fn = getattr(lib, nm)
        for _ in range(300):
            a, b, c, d = (rnd(rng, q[2 * k], q[2 * k + 1]) for k in range(4))
            fn(r, lv, U9(*a), U9(*b), U9(*c), U9(*d))
            check(r, lv)
            assert val(r) % P == (val(a) * val(b) + val(c) * val(d)) * RINV % P


def test_add_sub(lib):
    rng = random.Random(23)
    r, lv = U9(), I2()
    for sfx in ADDSUBS:
        La, Va, Lb, Vb = parse(sfx, 4)
        for op in ("add", "sub"):
            fn = getattr(lib, f"h_{op}_{sfx}")
            for _ in range(300):
                a, b = rnd(rng, La, Va), rnd(rng, Lb, Vb)
                fn(r, lv, U9(*a), U9(*b))
                check(r, lv)
                want = val(a) + val(b) if op == "add" else val(a) - val(b)
                assert (val(r) - want) % P == 0


def test_reduce_canon_normalize_neg(lib):
    rng = random.Random(24)
    r, lv = U9(), I2()
    cases = [rnd(rng, 8, 160) for _ in range(3000)]
    cases += [limbs(x) for x in (0, 1, P - 1, P, P + 1, 2 * P, 3 * P - 1, 3 * P, 159 * P, 160 * P - 1)]
    cases += [[8 * (2**29 - 1)] * 8 + [(160 * P - 1 - val([8 * (2**29 - 1)] * 8 + [0])) >> 232]]
    for a in cases:
        lib.h_reduce(r, lv, U9(*a))
        check(r, lv)
        assert lv[0] == 1 and lv[1] == 3 and (val(r) - val(a)) % P == 0
        lib.h_canon(r, lv, U9(*a))
        assert val(r) == val(a) % P and all(x < 2**29 for x in r)
        lib.h_normalize(r, lv, U9(*a))
        assert val(r) == val(a) and all(x < 2**29 for x in list(r)[:8])
    for _ in range(1000):
        b = rnd(rng, 6, 48)
        lib.h_neg(r, lv, U9(*b))
        check(r, lv)
        assert (val(r) + val(b)) % P == 0
        a = rnd(rng, 1, 16)
        lib.h_mul_small8(r, lv, U9(*a))
        check(r, lv)
        assert (val(r) - 8 * val(a)) % P == 0


def test_dot6_bounds_and_values(lib):
    rng = random.Random(28)
    r, lv = U9(), I2()
    U108 = ctypes.c_uint32 * 108
    for _ in range(400):
        xs = [rnd(rng, 1, 64) for _ in range(12)]
        lib.h_dot6(r, lv, U108(*sum(xs, [])))
        check(r, lv)
        want = sum(val(xs[2 * t]) * val(xs[2 * t + 1]) for t in range(6)) * RINV % P
        assert val(r) % P == want


def test_inverse(lib):
    rng = random.Random(25)
    r, lv = U9(), I2()
    for x in [1, 2, P - 1, 2**200] + [rng.randrange(1, P) for _ in range(200)]:
        a = limbs(x + P * rng.randrange(VS - 1))
        lib.h_inv(r, lv, U9(*a))
        check(r, lv)
        assert val(r) * val(a) % P == R * R % P  # (a R)^-1 in Montgomery form is a^-1 R
    lib.h_inv(r, lv, U9(*limbs(P)))
    assert val(r) % P == 0


# ---------------------------------------------------------------- the tower over plain integers
def f2mul(a, b):
    return ((a[0] * b[1] + a[1] * b[0]) % P, (a[1] * b[1] - a[0] * b[0]) % P)


def f2add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


XI = (1, 9)


def f6mul(a, b):
    # (x t^2 + y t + z)(x' t^2 + y' t + z'), t^3 = xi
    c = [(0, 0)] * 5
    A, B = (a[2], a[1], a[0]), (b[2], b[1], b[0])  # by ascending degree
    for i in range(3):
        for j in range(3):
            c[i + j] = f2add(c[i + j], f2mul(A[i], B[j]))
    c0 = f2add(c[0], f2mul(c[3], XI))
    c1 = f2add(c[1], f2mul(c[4], XI))
    return (c[2], c1, c0)


def f6pow(a, e):
    acc = ((0, 0), (0, 0), (0, 1))
    for bit in bin(e)[2:]:
        acc = f6mul(acc, acc)
        if bit == "1":
            acc = f6mul(acc, a)
    return acc


VS = None  # the stored value bound (bn254_fe9.cuh VS), read from the library


def enc2(rng, a):
    """a plain F_p^2 element -> stored limbs of its Montgomery form (value < VS p, random multiple)"""
    out = []
    for c in a:
        m = c * R % P + P * rng.randrange(VS - 1)
        out += limbs(m)
    return out


def dec2(l):
    return (val(l[0:9]) * RINV % P, val(l[9:18]) * RINV % P)


def enc6(rng, a):
    return enc2(rng, a[0]) + enc2(rng, a[1]) + enc2(rng, a[2])


def dec6(l):
    l = list(l)
    return (dec2(l[0:18]), dec2(l[18:36]), dec2(l[36:54]))


def stored(l):
    assert all(x < 2**29 for k, x in enumerate(l) if k % 9 != 8)
    for k in range(0, len(l), 9):
        assert val(l[k:k + 9]) < VS * P


def rnd2(rng):
    return (rng.randrange(P), rng.randrange(P))


def rnd6(rng):
    return (rnd2(rng), rnd2(rng), rnd2(rng))


def test_fp2(lib):
    rng = random.Random(26)
    U18 = ctypes.c_uint32 * 18
    r = U18()
    for _ in range(300):
        a, b = rnd2(rng), rnd2(rng)
        la, lb = U18(*enc2(rng, a)), U18(*enc2(rng, b))
        lib.h_fp2_mul(r, la, lb)
        stored(list(r))
        assert dec2(r) == f2mul(a, b)
        lib.h_fp2_sqr(r, la)
        stored(list(r))
        assert dec2(r) == f2mul(a, a)
        lib.h_fp2_mul_xi(r, la)
        stored(list(r))
        assert dec2(r) == f2mul(a, XI)
    for _ in range(40):
        a = rnd2(rng)
        lib.h_fp2_inv(r, U18(*enc2(rng, a)))
        assert f2mul(dec2(r), a) == (0, 1)


def test_fp6(lib):
    rng = random.Random(27)
    U54, U18 = ctypes.c_uint32 * 54, ctypes.c_uint32 * 18
    r = U54()
    for _ in range(100):
        a, b = rnd6(rng), rnd6(rng)
        la, lb = U54(*enc6(rng, a)), U54(*enc6(rng, b))
        lib.h_fp6_mul(r, la, lb)
        stored(list(r))
        assert dec6(r) == f6mul(a, b)
        lib.h_fp6_sqr(r, la)
        stored(list(r))
        assert dec6(r) == f6mul(a, a)
        y, z = rnd2(rng), rnd2(rng)
        lib.h_fp6_sparse(r, la, U18(*enc2(rng, y)), U18(*enc2(rng, z)))
        assert dec6(r) == f6mul(a, ((0, 0), y, z))
        lib.h_fp6_mul_tau(r, la)
        assert dec6(r) == f6mul(a, ((0, 0), (0, 1), (0, 0)))
    for _ in range(10):
        a = rnd6(rng)
        la = U54(*enc6(rng, a))
        lib.h_fp6_inv(r, la)
        assert f6mul(dec6(r), a) == ((0, 0), (0, 0), (0, 1))
    for _ in range(3):
        a = rnd6(rng)
        la = U54(*enc6(rng, a))
        ap = f6pow(a, P)
        lib.h_fp6_frob(r, la)
        assert dec6(r) == ap
        lib.h_fp6_frob_p2(r, la)
        assert dec6(r) == f6pow(ap, P)


def f6add(a, b):
    return tuple(f2add(x, y) for x, y in zip(a, b))


def test_fp6_lazy_operands(lib):
    rng = random.Random(29)
    U54, U18 = ctypes.c_uint32 * 54, ctypes.c_uint32 * 18
    r = U54()
    for _ in range(100):
        a, b, c, d = rnd6(rng), rnd6(rng), rnd6(rng), rnd6(rng)
        la, lb, lc, ld = (U54(*enc6(rng, v)) for v in (a, b, c, d))
        lib.h_fp6_mul_sums(r, la, lb, lc, ld)
        stored(list(r))
        assert dec6(r) == f6mul(f6add(a, b), f6add(c, d))
        y, z = rnd2(rng), rnd2(rng)
        lib.h_fp6_sparse_sum(r, la, lb, U18(*enc2(rng, y)), U18(*enc2(rng, z)))
        stored(list(r))
        assert dec6(r) == f6mul(f6add(a, b), ((0, 0), y, f2add(y, z)))
        lib.h_fp6_sub_tau(r, la, lb)
        stored(list(r))
        assert dec6(r) == f6add(f6mul(a, ((0, 0), (0, 1), (0, 0))), b)
