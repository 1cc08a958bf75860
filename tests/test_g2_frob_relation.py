"""The number theory behind the pairing path's G2 membership test (csrc/bn256.hip g2_frob_check).

The reference decides Q in G2 with Order*Q == infinity (crypto/bn256/cloudflare/twist.go:60-62).  The
GPU decides the same predicate from the point its line chain already ends on,
r = [6u+2]Q + psi(Q) - psi^2(Q) (optate.go:122-210): Q in G2 <=> r + psi^3(Q) == O.  These tests check
every number that argument rests on, and the relation itself on random points of E'(F_p^2) in G2, in
the cofactor part H and in neither, with plain Python integers (no GPU, no oracle).
"""
import math
import random

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583  # gfp.go p
N = 21888242871839275222246405745257275088548364400416034343698204186575808495617  # bn256.go Order
U = 4965661367192848881  # constants.go u
T = P + 1 - N  # trace of Frobenius
H = 2 * P - N  # #E'(F_p^2) / N
K = 6 * U + 2  # the Miller loop's length (sixuPlus2NAF)


def test_numbers():
    assert (K + P - P * P + P ** 3) % N == 0  # psi = [p] on G2: f(psi) kills G2
    assert math.gcd(N, H) == 1  # E'(F_p^2) = G2 x H
    # f(x) = x^3 - x^2 + x + K mod x^2 - T x + P = a + b x; its norm is coprime to h
    a, b = P + K - T * P, T * T - T - P + 1
    assert math.gcd(a * a + a * b * T + b * b * P, H) == 1
    # no addition in the chain meets +-Q for Q in G2 (the formulas would degenerate)
    for v in (K - P, K + P, K + P - P * P, K + P + P * P, K - 1, K + 1):
        assert v % N != 0


# F_p^2 = F_p[i] / (i^2 + 1), pairs (re, im)
def _add(x, y):
    return ((x[0] + y[0]) % P, (x[1] + y[1]) % P)


def _sub(x, y):
    return ((x[0] - y[0]) % P, (x[1] - y[1]) % P)


def _mul(x, y):
    return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)


def _inv(x):
    d = pow(x[0] * x[0] + x[1] * x[1], P - 2, P)
    return (x[0] * d % P, -x[1] * d % P)


def _pow(x, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = _mul(r, x)
        x = _mul(x, x)
        e >>= 1
    return r


XI = (9, 1)  # i + 9
TWIST_B = _mul((3, 0), _inv(XI))  # twist.go twistB = 3 / xi
C1, C2 = _pow(XI, (P - 1) // 3), _pow(XI, (P - 1) // 2)


def _sqrt(x):  # p = 3 mod 4
    a1 = _pow(x, (P - 3) // 4)
    alpha, x0 = _mul(a1, _mul(a1, x)), _mul(a1, x)
    r = _mul((0, 1), x0) if alpha == (P - 1, 0) else _mul(_pow(_add((1, 0), alpha), (P - 1) // 2), x0)
    return r if _mul(r, r) == x else None


def _padd(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    if p1[0] == p2[0]:
        if p1[1] != p2[1] or p1[1] == (0, 0):
            return None
        lam = _mul(_mul((3, 0), _mul(p1[0], p1[0])), _inv(_mul((2, 0), p1[1])))
    else:
        lam = _mul(_sub(p2[1], p1[1]), _inv(_sub(p2[0], p1[0])))
    x3 = _sub(_sub(_mul(lam, lam), p1[0]), p2[0])
    return (x3, _sub(_mul(lam, _sub(p1[0], x3)), p1[1]))


def _neg(q):
    return None if q is None else (q[0], ((-q[1][0]) % P, (-q[1][1]) % P))


def _smul(k, q):
    if k < 0:
        return _smul(-k, _neg(q))
    r = None
    while k:
        if k & 1:
            r = _padd(r, q)
        q = _padd(q, q)
        k >>= 1
    return r


def _psi(q):  # optate.go:173-176 on affine points
    conj = lambda x: (x[0], (-x[1]) % P)
    return None if q is None else (_mul(conj(q[0]), C1), _mul(conj(q[1]), C2))


def _f(q):  # r + psi^3(Q) with r the line chain's final point
    r = _padd(_padd(_smul(K, q), _psi(q)), _neg(_psi(_psi(q))))
    return _padd(r, _psi(_psi(_psi(q))))


def test_relation_on_random_points():
    rng = random.Random(7)
    for _ in range(2):
        while True:
            x = (rng.randrange(P), rng.randrange(P))
            y = _sqrt(_add(_mul(x, _mul(x, x)), TWIST_B))
            if y:
                break
        q = (x, y)
        assert _smul(N * H, q) is None
        assert _padd(_padd(_psi(_psi(q)), _smul(-T, _psi(q))), _smul(P, q)) is None  # psi^2 - t psi + p = 0
        g, h = _smul(H, q), _smul(N, q)  # in G2, in H
        assert _smul(N, g) is None and _f(g) is None
        assert _smul(N, q) is not None and _f(q) is not None
        assert h is not None and _f(h) is not None
