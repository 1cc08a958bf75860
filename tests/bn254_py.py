"""TEST INFRASTRUCTURE — small pure-Python BN254 helpers, independent of the C oracle.

Affine group law on G1 (y^2 = x^3 + 3 over F_p) and on the sextic twist
(y^2 = x^3 + 3/xi over F_p^2, xi = 9 + i), plus an F_p^2 square root.  Used to build
precompile inputs with a known class (off-curve, on the twist but outside the order-r
subgroup, ...) and to confirm that class without going through the oracle under test.
Parameters: crypto/bn256/cloudflare/constants.go:17-23, curve.go:14, twist.go:15-18.
Encoding: core/vm/contracts.go:256-272 / bn256.go:256-306 (G2 imaginary part first).
"""
from __future__ import annotations

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617


# F_p^2 elements as (re, im) = re + im*i, i^2 = -1
def f2(a, b=0):
    return (a % P, b % P)


def add2(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def sub2(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def mul2(a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % P, (a[0] * b[1] + a[1] * b[0]) % P)


def inv2(a):
    n = (a[0] * a[0] + a[1] * a[1]) % P
    ni = pow(n, P - 2, P)
    return (a[0] * ni % P, (-a[1]) * ni % P)


def pow2(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = mul2(r, a)
        a = mul2(a, a)
        e >>= 1
    return r


def sqrt2(a):
    """square root in F_p^2 (p = 3 mod 4), or None"""
    if a == (0, 0):
        return (0, 0)
    a1 = pow2(a, (P - 3) // 4)
    alpha = mul2(a1, mul2(a1, a))
    a0 = mul2(pow2(alpha, P), alpha)
    if a0 == (P - 1, 0):
        return None
    x0 = mul2(a1, a)
    if alpha == (P - 1, 0):
        x = mul2((0, 1), x0)
    else:
        b = pow2(add2((1, 0), alpha), (P - 1) // 2)
        x = mul2(b, x0)
    return x if mul2(x, x) == a else None


TWIST_B = mul2(f2(3), inv2(f2(9, 1)))


def g2_on_twist(x, y):
    return mul2(y, y) == add2(mul2(mul2(x, x), x), TWIST_B)


def g2_add(p, q):
    """affine addition on the twist; None = infinity"""
    if p is None:
        return q
    if q is None:
        return p
    (x1, y1), (x2, y2) = p, q
    if x1 == x2:
        if add2(y1, y2) == (0, 0):
            return None
        lam = mul2(mul2(f2(3), mul2(x1, x1)), inv2(add2(y1, y1)))
    else:
        lam = mul2(sub2(y2, y1), inv2(sub2(x2, x1)))
    x3 = sub2(sub2(mul2(lam, lam), x1), x2)
    y3 = sub2(mul2(lam, sub2(x1, x3)), y1)
    return (x3, y3)


def g2_mul(p, k):
    r = None
    while k:
        if k & 1:
            r = g2_add(r, p)
        p = g2_add(p, p)
        k >>= 1
    return r


def g2_encode(p) -> bytes:
    if p is None:
        return bytes(128)
    (x, y) = p
    return b"".join(v.to_bytes(32, "big") for v in (x[1], x[0], y[1], y[0]))


def g2_decode(b: bytes):
    v = [int.from_bytes(b[32 * i:32 * i + 32], "big") for i in range(4)]
    if v == [0, 0, 0, 0]:
        return None
    return ((v[1], v[0]), (v[3], v[2]))


def twist_point_outside_g2(seed: int):
    """a point on the twist E'(F_p^2) that is NOT in the order-r subgroup G2"""
    x0 = seed
    while True:
        x = f2(x0, x0 * 7 + 1)
        y = sqrt2(add2(mul2(mul2(x, x), x), TWIST_B))
        if y is not None:
            pt = (x, y)
            assert g2_on_twist(*pt)
            if g2_mul(pt, R) is not None:
                return pt
        x0 += 1


def g1_on_curve(x, y):
    return (y * y - x * x * x - 3) % P == 0
