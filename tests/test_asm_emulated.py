"""The generated inline-asm field operations (tools/gen_fe9_asm.py -> csrc/fe9_asm.cuh,
tools/gen_bn9_asm.py -> csrc/bn9_asm.cuh), executed instruction by instruction on the CPU.

Each instruction's gfx950 semantics are restated below and every 64-bit multiply-add, shift-add
and 32-bit add is checked not to wrap, at the extreme limb and value bounds the C++ callers admit
(secp256k1_fe9.cuh magnitudes; bn254_fe9.cuh fqm<L, V> bounds).  The results are checked against
Python integers: a*b mod p (secp256k1, weakly normalised) and sum(a_t b_t) R^-1 mod p (BN254,
R = 2^261).  The GPU tests then check the same code bit-exact against the oracle."""
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_bn9_asm  # noqa: E402
import gen_fe9_asm  # noqa: E402

M32, M64 = (1 << 32) - 1, (1 << 64) - 1
P_SECP = 2**256 - 2**32 - 977


def _bn_p():
    # bn256 cloudflare P (crypto/bn256/cloudflare/constants.go): 36u^4 + 36u^3 + 24u^2 + 6u + 1
    u = 4965661367192848881
    return 36 * u**4 + 36 * u**3 + 24 * u**2 + 6 * u + 1


P_BN = _bn_p()


class Machine:
    """Operand slots (%N) and physical VGPRs; 64-bit operands are physical pairs v[a:b]."""

    def __init__(self, ops):
        self.ops = dict(ops)
        self.v = {}

    def r32(self, x):
        if x.startswith("%"):
            return self.ops[int(x[1:])]
        if x.startswith("v"):
            return self.v[int(x[1:])]
        return int(x, 0)

    def r64(self, x):
        if x.startswith("v["):
            lo, hi = (int(t) for t in x[2:-1].split(":"))
            return self.v[lo] | (self.v[hi] << 32)
        assert not x.startswith("%"), x
        return int(x, 0)

    def w32(self, x, val):
        assert 0 <= val <= M32
        if x.startswith("%"):
            self.ops[int(x[1:])] = val
        else:
            self.v[int(x[1:])] = val

    def w64(self, x, val):
        assert 0 <= val <= M64
        if x.startswith("%"):
            return  # the dead carry-out SGPR pair
        lo, hi = (int(t) for t in x[2:-1].split(":"))
        self.v[lo], self.v[hi] = val & M32, val >> 32

    def run(self, lines):
        for ln in lines:
            op, rest = ln.split(" ", 1)
            a = [t.strip() for t in rest.split(",")]
            if op == "v_mad_u64_u32":
                res = self.r32(a[2]) * self.r32(a[3]) + self.r64(a[4])
                assert res <= M64, f"64-bit overflow in {ln}"
                self.w64(a[0], res)
            elif op == "v_lshrrev_b64":
                self.w64(a[0], self.r64(a[2]) >> int(a[1]))
            elif op == "v_lshlrev_b64":
                self.w64(a[0], (self.r64(a[2]) << int(a[1])) & M64)
            elif op == "v_lshl_add_u64":
                assert 0 <= int(a[2]) <= 4, f"v_lshl_add_u64 shifts by 0..4 only: {ln}"
                res = (self.r64(a[1]) << int(a[2])) + self.r64(a[3])
                assert res <= M64, f"64-bit overflow in {ln}"
                self.w64(a[0], res)
            elif op == "v_lshlrev_b32":
                res = self.r32(a[2]) << int(a[1])
                assert res <= M32, f"32-bit shift loses bits in {ln}"
                self.w32(a[0], res)
            elif op == "v_and_b32_e32":
                self.w32(a[0], int(a[1], 0) & self.r32(a[2]))
            elif op == "v_mov_b32":
                self.w32(a[0], self.r32(a[1]))
            elif op == "v_add_u32":
                res = self.r32(a[1]) + self.r32(a[2])
                assert res <= M32, f"32-bit overflow in {ln}"
                self.w32(a[0], res)
            elif op == "v_add3_u32":
                res = self.r32(a[1]) + self.r32(a[2]) + self.r32(a[3])
                assert res <= M32, f"32-bit overflow in {ln}"
                self.w32(a[0], res)
            elif op == "v_mad_u32_u24":
                x, y = self.r32(a[1]), self.r32(a[2])
                assert x < 1 << 24 and y < 1 << 24, f"u24 operand out of range in {ln}"
                res = x * y + self.r32(a[3])
                assert res <= M32, f"32-bit overflow in {ln}"
                self.w32(a[0], res)
            elif op == "v_alignbit_b32":
                self.w32(a[0], (((self.r32(a[1]) << 32) | self.r32(a[2])) >> int(a[3])) & M32)
            elif op == "v_mul_lo_u32":
                self.w32(a[0], (self.r32(a[1]) * self.r32(a[2])) & M32)
            else:
                raise AssertionError(f"no semantics for {op}")


def limbs_val(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def to_limbs(v, n=9):
    return [(v >> (29 * i)) & ((1 << 29) - 1) for i in range(n - 1)] + [v >> (29 * (n - 1))]


def redundant(limbs, mag, rng):
    """the same value with limbs pushed up to < mag * 2^29 by borrowing from the next limb"""
    l = list(limbs)
    for i in range(8):
        room = int(mag * (1 << 29)) - 1 - l[i]
        k = min(room >> 29, l[i + 1])
        if k > 0:
            k = rng.randint(0, k) if rng.random() < 0.5 else k
            l[i] += k << 29
            l[i + 1] -= k
    return l


# --------------------------------------------------------------------------- secp256k1 fe9
def fe9_case(rng, ma, mb, extreme):
    lim = lambda m: [int(m * (1 << 29)) - 1] * 8 + [min(int(m * (1 << 24)) - 1, M32)]
    if extreme:
        return lim(ma), lim(mb)
    a = redundant(to_limbs(rng.randrange(P_SECP)), ma, rng)
    b = redundant(to_limbs(rng.randrange(P_SECP)), mb, rng)
    return a, b


OPND1 = {"r": 0, "a": 18, "b": 27, "k31264": 36, "k256": 37, "k977": 38, "c": 39, "d": 48}
# the column forms of tools/gen_fe9_asm.py (GSV_FE9_COLS 1 / 2 / 3) and their operand numbering
FORMS = {1: (gen_fe9_asm.full_lines, OPND1), 2: (gen_fe9_asm.full_lines2, gen_fe9_asm.OPND2),
         3: (gen_fe9_asm.full_lines3, gen_fe9_asm.OPND2)}


def fe9_lines(form, terms, addend=False):
    gen, lay = FORMS[form]
    return (gen(terms, addend), lay)


def run_fe9(lines, a, b, c=None, d=None):
    lines, O = lines
    ops = {O["a"] + i: a[i] for i in range(9)}
    ops.update({O["b"] + j: b[j] for j in range(9)})
    if c is not None:
        ops.update({O["c"] + j: c[j] for j in range(9)})
    if d is not None:
        ops.update({O["d"] + j: d[j] for j in range(9)})
    ops.update({O["k31264"]: 31264, O["k256"]: 256, O["k977"]: 977})
    if "k8192" in O:
        ops[O["k8192"]] = 8192
    m = Machine(ops)
    m.run(lines)
    return [m.ops[O["r"] + i] for i in range(9)]


def check_weak(r, want):
    assert limbs_val(r) % P_SECP == want % P_SECP
    assert all(r[i] < (1 << 29) for i in (0, 1, 3, 4, 5, 6, 7)) and r[2] <= (1 << 29) + (1 << 24) and r[8] < (1 << 24)


@pytest.mark.parametrize("ma,mb", [(1, 1), (1, 7), (7, 1), (2.64, 2.64), (2, 3.5)])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_mul_asm(form, ma, mb):
    rng = random.Random(int(ma * 100 + mb))
    lines = fe9_lines(form, gen_fe9_asm.MUL_TERMS)
    for it in range(150):
        a, b = fe9_case(rng, ma, mb, extreme=(it == 0))
        check_weak(run_fe9(lines, a, b), limbs_val(a) * limbs_val(b))


@pytest.mark.parametrize("ma", [1, 2, 2.64])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_sqr_asm(form, ma):
    rng = random.Random(int(ma * 100))
    lines = fe9_lines(form, gen_fe9_asm.SQR_TERMS)
    for it in range(150):
        a, _ = fe9_case(rng, ma, 1, extreme=(it == 0))
        a2 = [x << 1 for x in a]
        assert max(a2) <= M32
        check_weak(run_fe9(lines, a, a2), limbs_val(a) ** 2)


Q3_MAX = [(4 << 29) - 1] * 8 + [(4 << 29) - 1]  # fe9_negsum<3> addend limbs: Q_3 limbs < 2^31


def addend_case(rng, extreme):
    """c of fe9_mul_add / fe9_sqr_add: Q_M - x - y (- z), M <= 3: every limb in [0, 2^31)"""
    if extreme:
        return list(Q3_MAX)
    return [rng.randrange(1 << 31) for _ in range(9)]


@pytest.mark.parametrize("ma,mb", [(1.04, 1.04), (1, 3), (1.04, 4.16), (1, 7)])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_mul_add_asm(form, ma, mb):
    rng = random.Random(int(ma * 1000 + mb))
    lines = fe9_lines(form, gen_fe9_asm.MUL_TERMS, addend=True)
    for it in range(150):
        a, b = fe9_case(rng, ma, mb, extreme=(it == 0))
        c = addend_case(rng, extreme=(it < 2))
        check_weak(run_fe9(lines, a, b, c), limbs_val(a) * limbs_val(b) + limbs_val(c))


@pytest.mark.parametrize("ma", [1, 1.04, 2.64])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_sqr_add_asm(form, ma):
    rng = random.Random(int(ma * 1000) + 7)
    lines = fe9_lines(form, gen_fe9_asm.SQR_TERMS, addend=True)
    for it in range(150):
        a, _ = fe9_case(rng, ma, 1, extreme=(it == 0))
        a2 = [x << 1 for x in a]
        c = addend_case(rng, extreme=(it < 2))
        check_weak(run_fe9(lines, a, a2, c), limbs_val(a) ** 2 + limbs_val(c))


@pytest.mark.parametrize("m", [(1.04, 3.04, 1.04, 3), (1, 3.5, 1, 3.5), (1.04, 1.04, 2.64, 2.2)])
@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_dot_asm(form, m):
    """a*b + c*d with one reduction at m_a m_b + m_c m_d <= 7 (the mixed add's Y3: rr (V - X3) + Y1 (-2J))"""
    ma, mb, mc, md = m
    rng = random.Random(int(sum(m) * 1000))
    lines = fe9_lines(form, gen_fe9_asm.DOT_TERMS)
    for it in range(150):
        a, b = fe9_case(rng, ma, mb, extreme=(it == 0))
        c, d = fe9_case(rng, mc, md, extreme=(it == 0))
        check_weak(run_fe9(lines, a, b, c, d), limbs_val(a) * limbs_val(b) + limbs_val(c) * limbs_val(d))


def _q_consts():
    """FE9_Q[M] limbs from fe9_q_consts.inc (Q_1..Q_7)"""
    src = open(os.path.join(ROOT, "geth-sharding_amd", "csrc", "fe9_q_consts.inc")).read()
    rows = [r for r in src.split("\n") if r.strip().startswith("{")]
    return {m + 1: [int(x.strip().rstrip("u"), 16) for x in rows[m].strip().strip("{},").split(",")] for m in range(7)}


@pytest.mark.parametrize("form", [1, 2, 3])
def test_fe9_dot_asm_at_the_mixed_add_operands(form):
    """the operands fe9_dot actually gets in gej9_add_ge_core, at their largest limbs: rr and Y1 are
    product outputs (limb 2 up to 2^29 + 2^24), V - X3 = V + (Q_1 - X3), -2J = Q_2 - J - J (limb 8
    near 2^30, far above a product output's 2^24)"""
    Q = _q_consts()
    prod = [(1 << 29) - 1] * 9
    prod[2] = (1 << 29) + (1 << 24) - 1
    prod[8] = (1 << 24) - 1
    t = [prod[i] + Q[1][i] for i in range(9)]      # V - X3 with X3 = 0
    w = list(Q[2])                                 # -2J with J = 0
    lines = fe9_lines(form, gen_fe9_asm.DOT_TERMS)
    check_weak(run_fe9(lines, prod, t, prod, w), limbs_val(prod) * limbs_val(t) + limbs_val(prod) * limbs_val(w))
    rng = random.Random(99)
    for _ in range(200):
        a = [rng.randrange(x + 1) for x in prod]
        c = [rng.randrange(x + 1) for x in prod]
        b = [rng.randrange(x + 1) for x in t]
        d = [rng.randrange(x + 1) for x in w]
        check_weak(run_fe9(lines, a, b, c, d), limbs_val(a) * limbs_val(b) + limbs_val(c) * limbs_val(d))


# --------------------------------------------------------------------------- BN254 REDC
FQ_M = (1 << 29) - 1
R_BN = 1 << 261
FQ_PROD_MAX = 168 * (160 - 2)


def bn_p_limbs():
    return to_limbs(P_BN)


def run_redc(N, A, B):
    lines = gen_bn9_asm.redc_lines(N)
    ops = {}
    for t in range(N):
        for i in range(9):
            ops[19 + 9 * t + i] = A[t][i]
            ops[19 + 9 * N + 9 * t + i] = B[t][i]
    pl = bn_p_limbs()
    for j in range(9):
        ops[19 + 18 * N + j] = pl[j]
    ops[19 + 18 * N + 9] = (-pow(P_BN, -1, 1 << 29)) % (1 << 29)
    m = Machine(ops)
    m.run(lines)
    return [m.ops[i] for i in range(9)]


# (L, V) bounds per product: sum La Lb <= 6 and sum Va Vb <= FQ_PROD_MAX (bn254_fe9.cuh fq_dot)
BN_CASES = [
    [((1, 20), (1, 20))],
    [((6, 160), (1, 160))],
    [((2, 100), (3, 100))],
    [((1, 20), (1, 20)), ((1, 20), (1, 20))],
    [((2, 80), (1, 80)), ((2, 80), (2, 80))],
    [((1, 60), (1, 60))] * 3,
    [((1, 40), (1, 40))] * 4,
    [((1, 20), (1, 20))] * 5,
    [((1, 20), (1, 20))] * 6,
]


@pytest.mark.parametrize("case", BN_CASES, ids=lambda c: f"N{len(c)}")
def test_bn_redc_asm(case):
    N = len(case)
    assert sum(la * lb for ((la, _), (lb, _)) in case) <= 6
    assert sum(va * vb for ((_, va), (_, vb)) in case) <= FQ_PROD_MAX
    rng = random.Random(N * 1000 + case[0][0][0])
    vbound = sum(va * vb for ((_, va), (_, vb)) in case) // 168 + 2
    for it in range(100):
        A, B = [], []
        for ((la, va), (lb, vb)) in case:
            for (L, V, dst) in ((la, va, A), (lb, vb, B)):
                x = V * P_BN - 1 if it == 0 else rng.randrange(V * P_BN)
                limbs = redundant(to_limbs(x), L, rng) if x < (1 << 261) else None
                if limbs is None or limbs[8] > L * FQ_M:
                    x = rng.randrange(min(V * P_BN, 1 << 261))
                    limbs = redundant(to_limbs(x), L, rng)
                assert all(l <= L * FQ_M for l in limbs)
                dst.append(limbs)
        r = run_redc(N, A, B)
        T = sum(limbs_val(A[t]) * limbs_val(B[t]) for t in range(N))
        assert (limbs_val(r) * R_BN - T) % P_BN == 0
        assert all(x < (1 << 29) for x in r[:8])
        assert limbs_val(r) < vbound * P_BN
