"""The twisted-curve recovery tail of csrc/recover_dev.cuh (GSV_RECOVER_TWIST, recover_tail_twisted),
restated with Python integers and checked against affine arithmetic on secp256k1: u2 R computed on
E_t: y^2 = x^3 + 7 c^3 from R* = (c x, c^2) (no square root), the sum with u1 G carried as a + t b with
t = y_R, and one exponentiation w = (c z^4)^((p-3)/4) giving both the root and the inverse of Z.
Covers u1 G = O, u1 G = u2 R (doubling), u1 G = -u2 R (infinity: recovery fails) and non-square
c = x^3 + 7 (no R: recovery fails), the failure classes of libsecp256k1's recovery
(crypto/secp256k1/libsecp256k1/src/modules/recovery/main_impl.h:87-121)."""
import random

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
E_PM3_4 = (P - 3) // 4


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], P - 2, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], P - 2, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return x, (lam * (a[0] - x) - a[1]) % P


def _mul(k, pt):  # any a = 0 curve: the formulas do not involve b
    r = None
    while k:
        if k & 1:
            r = _add(r, pt)
        pt = _add(pt, pt)
        k >>= 1
    return r


def _jac(pt, rng):
    z = rng.randrange(1, P)
    return pt[0] * z * z % P, pt[1] * z ** 3 % P, z


def _dbl_jac(pt):  # gej9_dbl
    x, y, z = pt
    a, b = x * x, y * y
    d, e = 4 * x * b, 3 * a
    x3 = (e * e - 2 * d) % P
    return x3, (e * (d - x3) - 8 * b * b) % P, 2 * y * z % P


def tail(x, par, p1, p2):
    """recover_tail_twisted: p1 = u1 G (Jacobian on E or None), p2 = u2 R* (Jacobian on E_t)"""
    c = (x ** 3 + 7) % P
    xs, ys, zs = p2
    exc = False
    if p1 is None:
        x3a, db, y3a, y3b, z = xs, 0, ys, 0, zs
    else:
        x1, y1, z1 = p1
        z1z1, z2z2 = z1 * z1 % P, c * zs * zs % P
        u1 = x1 * z2z2 % P
        h = (xs * z1z1 - u1) % P
        s1p = y1 * zs * z2z2 % P
        s2 = ys * z1 * z1z1 % P
        exc = h == 0
        if exc:
            x3a, y3a, z = _dbl_jac(p2)
            db, y3b = s1p, s2
        else:
            hh = h * h % P
            hhh, v = h * hh % P, u1 * hh % P
            x3a = (s2 * s2 + c * s1p * s1p - hhh - 2 * v) % P
            db = 2 * s2 * s1p % P
            da = (v - x3a) % P
            y3a = (s2 * da - c * s1p * db) % P
            y3b = (s2 * db - s1p * (da + hhh)) % P
            z = z1 * zs * h % P
    w = pow(c * pow(z, 4, P) % P, E_PM3_4, P)
    m = w * z % P
    s0 = c * m * z % P
    if s0 * s0 % P != c:
        return "fail"
    flip = (s0 & 1) != par
    pb, qb = s0 * db % P, s0 * y3b % P
    if exc:
        rr = (y3b + pb) if flip else (y3b - pb)
        if rr % P:
            return "fail"
        pb = qb = 0
    xq = (x3a + (pb if flip else -pb)) * m * m % P
    yq = ((-y3a if flip else y3a) + qb) * m ** 3 % P
    return xq, yq


def _sqrt(a):
    r = pow(a, (P + 1) // 4, P)
    return r if r * r % P == a % P else None


def test_chain_exponent_bits():
    # fe9_pow_pm3_4's chain: [223 ones] 0 [22 ones] 0000 1 0 11
    want = "1" * 223 + "0" + "1" * 22 + "0000" + "1" + "0" + "11"
    assert bin(E_PM3_4)[2:] == want


def test_tail_matches_affine_sum():
    rng = random.Random(7)
    for it in range(60):
        while True:
            x = rng.randrange(P)
            y = _sqrt(x ** 3 + 7)
            if y is not None:
                break
        par = rng.randrange(2)
        if (y & 1) != par:
            y = P - y
        R = (x, y)
        u2 = rng.randrange(1, N)
        u1 = 0 if it % 5 == 1 else rng.randrange(1, N)
        p1 = _mul(u1, G)
        if it % 5 == 2:
            p1 = _mul(u2, R)                      # u1 G == u2 R: the doubling
        if it % 5 == 3:
            t = _mul(u2, R)
            p1 = (t[0], (-t[1]) % P)              # u1 G == -u2 R: infinity
        c = (x ** 3 + 7) % P
        p2 = _jac(_mul(u2, (c * x % P, c * c % P)), rng)
        want = _add(p1, _mul(u2, R))
        got = tail(x, par, _jac(p1, rng) if p1 else None, p2)
        assert got == (want if want is not None else "fail"), it


def test_tail_rejects_non_square():
    rng = random.Random(8)
    seen = 0
    while seen < 20:
        x = rng.randrange(P)
        if _sqrt(x ** 3 + 7) is not None:
            continue
        seen += 1
        c = (x ** 3 + 7) % P
        p2 = _jac(_mul(5, (c * x % P, c * c % P)), rng)   # a point of the twist
        assert tail(x, 0, _jac(G, rng), p2) == "fail"
