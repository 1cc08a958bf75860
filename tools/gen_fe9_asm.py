"""Generates geth-sharding_amd/csrc/fe9_asm.cuh: secp256k1_fe9.cuh's fe9_mul / fe9_sqr (9 x 29-bit
column product + the 2^261 == 2^37 + 31264 fold of fe9_reduce) as ONE inline-asm statement each.

Why asm.  Written as C++ (`acc += (uint64_t)a[i] * b[j]` per term, `acc >>= 29` per column),
LLVM re-associates each column's sum into a v_mad_u64_u32 chain that starts at 0 and adds the
incoming carry with a separate v_lshl_add_u64 (17 extra 64-bit VALU ops per product, 8 more in
the reduction).  Pinning the order with an empty asm after every multiply-add removes those, but
hipcc then pads a wait state (s_nop 0) after every asm boundary whose output the next VALU reads:
73 per product.  One statement for the whole operation has neither: column k's accumulator
starts as the previous column shifted right by 29 (v_lshrrev_b64) and takes its products as one
chain; the reduction's running value keeps its carry in a register pair whose high word is 0.

Inline asm cannot name the low half of a 64-bit operand, so the two running pairs live in fixed,
clobbered VGPRs (v[2:3], v[4:5]) and the 29-bit limbs are read from their low registers.
full_lines() is also executed instruction by instruction by tests/test_asm_emulated.py."""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "geth-sharding_amd", "csrc", "fe9_asm.cuh")


def full(name, doc, terms_of_column, addend=False, dot=False):
    L = full_lines(terms_of_column, addend)
    outs = ", ".join([f'"=&v"(r[{i}])' for i in range(9)] + [f'"=&v"(hi[{i}])' for i in range(8)] + ['"=&s"(sd)'])
    ins = ", ".join([f'"v"(a[{i}])' for i in range(9)] + [f'"v"(b[{j}])' for j in range(9)] +
                    ['"s"(k31264)', '"s"(k256)', '"s"(k977)'] +
                    ([f'"v"(c[{j}])' for j in range(9)] if addend or dot else []) +
                    ([f'"v"(d[{j}])' for j in range(9)] if dot else []))
    body = "\\n\\t".join(L)
    return [f"// {doc}",
            f"__device__ __forceinline__ void {name}(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]"
            + (", const uint32_t c[9]" if addend or dot else "") + (", const uint32_t d[9]" if dot else "") + ") {",
            "    uint32_t hi[8];",
            "    uint64_t sd;",
            "    uint32_t k31264 = 31264u, k256 = 256u, k977 = 977u;",
            f'    asm("{body}"',
            f"        : {outs}",
            f"        : {ins}",
            '        : "v2", "v3", "v4", "v5");',
            "}"]


MUL_TERMS = lambda k: [(i, 9 + (k - i)) for i in range(9) if 0 <= k - i < 9]


def DOT_TERMS(k):
    """a b + c d: both products' terms in one column chain (one reduction for the two)"""
    return MUL_TERMS(k) + [(18 + i, 27 + (k - i)) for i in range(9) if 0 <= k - i < 9]


def SQR_TERMS(k):
    """squaring: b holds the doubled limbs 2 a[j]; cross terms a[i] * 2a[j] (i < j) + a[k/2]^2"""
    t = [(i, 9 + (k - i)) for i in range(9) if i < k - i < 9]
    if k % 2 == 0 and k // 2 < 9:
        t.append((k // 2, k // 2))
    return t


def full_lines(terms_of_column, addend=False):
    """Product + reduction (secp256k1_fe9.cuh fe9_reduce restated) in one statement.  Operands:
    %0..%8 r (o_0..o_8 in place), %9..%16 o_9..o_16, %17 sd, %18..%26 a, %27..%35 b,
    %36 31264, %37 256, %38 977 (SGPRs), with `addend` %39..%47 the limbs of c (each < 2^31),
    added to o_0..o_8 as the reduction reads them (r = a b + c; the 32-bit add that takes o_j becomes
    a three-operand add, no further instruction).  Fixed pairs: C = v[2:3] (columns, then o17, then
    T), D = v[4:5] (the reduction's running value)."""
    cj = lambda j: f"%{39 + j}"
    # term operand numbering: 0..8 a, 9..17 b, 18..26 c (%39..), 27..35 d (%48..; fe9_dot only)
    opnd = lambda x: f"%{18 + x}" if x < 18 else f"%{39 + (x - 18)}"
    C, c0, c1 = "v[2:3]", "v2", "v3"
    D, d0, d1 = "v[4:5]", "v4", "v5"
    o = lambda k: f"%{k}" if k < 9 else f"%{k}"
    a = lambda i: f"%{18 + i}"
    b = lambda j: f"%{27 + j}"
    K31264, K256, K977, SD = "%36", "%37", "%38", "%17"
    L = []
    for k in range(17):
        first = True
        if k > 0:
            L.append(f"v_lshrrev_b64 {C}, 29, {C}")
            first = False
        for (x, y) in terms_of_column(k):
            L.append(f"v_mad_u64_u32 {C}, {SD}, {opnd(x)}, {opnd(y)}, {'0' if first else C}")
            first = False
        L.append(f"v_and_b32_e32 {o(k)}, 0x1fffffff, {c0}")
    L.append(f"v_lshrrev_b64 {C}, 29, {C}")               # o17 < 2^35
    # limbs 0..7: c = o_j + carry + 31264 o_{j+9} + 256 o_{j+8}
    L.append(f"v_mov_b32 {d1}, 0")
    if addend:
        L.append(f"v_add_u32 {d0}, {o(0)}, {cj(0)}")       # o_0 + c_0 < 2^29 + 2^31
    else:
        L.append(f"v_mov_b32 {d0}, {o(0)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {o(9)}, {K31264}, {D}")
    L.append(f"v_and_b32_e32 {o(0)}, 0x1fffffff, {d0}")
    for j in range(1, 8):
        L.append(f"v_lshrrev_b64 {D}, 29, {D}")           # carry < 2^17: the high word is 0
        if addend:
            L.append(f"v_add3_u32 {d0}, {d0}, {o(j)}, {cj(j)}")
        else:
            L.append(f"v_add_u32 {d0}, {d0}, {o(j)}")
        L.append(f"v_mad_u64_u32 {D}, {SD}, {o(j + 9)}, {K31264}, {D}")
        L.append(f"v_mad_u64_u32 {D}, {SD}, {o(j + 8)}, {K256}, {D}")
        L.append(f"v_and_b32_e32 {o(j)}, 0x1fffffff, {d0}")
    # limb 8: o_8 + carry + 31264 o17 + 256 o_16; 24 bits stay, the rest (units of 2^256) is T
    L.append(f"v_lshrrev_b64 {D}, 29, {D}")
    if addend:
        L.append(f"v_add3_u32 {d0}, {d0}, {o(8)}, {cj(8)}")
    else:
        L.append(f"v_add_u32 {d0}, {d0}, {o(8)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {c0}, {K31264}, {D}")
    L.append(f"v_mad_u32_u24 {d1}, {c1}, {K31264}, {d1}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {o(16)}, {K256}, {D}")
    L.append(f"v_and_b32_e32 {o(8)}, 0xffffff, {d0}")
    L.append(f"v_lshrrev_b64 {D}, 24, {D}")
    L.append(f"v_lshlrev_b64 {C}, 13, {C}")             # (v_lshl_add_u64 shifts by 0..4 only)
    L.append(f"v_lshl_add_u64 {C}, {C}, 0, {D}")        # T = (c >> 24) + (o17 << 13) < 2^49
    # 2^256 == 2^32 + 977: limb 0 += 977 T, limb 1 += 8 T (+ carries), limb 2 += carry
    L.append(f"v_mov_b32 {d1}, 0")
    L.append(f"v_mov_b32 {d0}, {o(0)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {c0}, {K977}, {D}")
    L.append(f"v_mad_u32_u24 {d1}, {c1}, {K977}, {d1}")
    L.append(f"v_and_b32_e32 {o(0)}, 0x1fffffff, {d0}")
    L.append(f"v_lshrrev_b64 {D}, 29, {D}")
    L.append(f"v_lshl_add_u64 {D}, {C}, 3, {D}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {o(1)}, 1, {D}")
    L.append(f"v_and_b32_e32 {o(1)}, 0x1fffffff, {d0}")
    L.append(f"v_alignbit_b32 {c0}, {d1}, {d0}, 29")
    L.append(f"v_add_u32 {o(2)}, {o(2)}, {c0}")
    return L



# ---------------------------------------------------------------------------- column form 2
# Operand numbering of the form-2 statements (the emulator test reads it): %0..%8 r, %9 the dead
# carry-out SGPR pair, then a, b, the three SGPR constants, c, d.
OPND2 = {"r": 0, "sd": 9, "a": 10, "b": 19, "k31264": 28, "k256": 29, "k977": 30, "k8192": 31, "c": 32, "d": 41}
PAIR2 = {k: f"v[{6 + 2 * (k - 10)}:{7 + 2 * (k - 10)}]" for k in range(10, 17)}  # columns 10..16


def full_lines2(terms_of_column, addend=False):
    """Form 2: the high columns 9..16 are never masked or shifted.  Column 9 accumulates in
    C = v[2:3] (from column 8's C >> 29, as form 1); column k = 10..16 in its own fixed pair P_k
    (v[6:7] .. v[18:19]) starting from 8 * hi(P_{k-1}) (one multiply-add, in place of the 64-bit shift)
    and keeps its 32-bit low word o_k = C_k mod 2^32 unmasked: sum_k o_k 2^(29 k) is still the product,
    because the carry into column k is floor(C_{k-1} / 2^32) at weight 2^(29 (k-1) + 32) = 8 * 2^(29 k).
    The reduction reads o_9..o_16 through multiply-adds (31264 o, 256 o < 2^47), so an unmasked 32-bit
    limb costs nothing there; o17 = 8 hi(P_16) < 2^23 is a 32-bit value (one shift), and
    T = (c >> 24) + o17 2^13 one multiply-add.  Per product 8 masks, a 64-bit shift, a 64-bit
    shift-add and a u24 multiply-add fewer than form 1."""
    O = OPND2
    opnd = lambda x: f"%{O['a'] + x}" if x < 9 else (f"%{O['b'] + x - 9}" if x < 18 else f"%{O['c'] + x - 18}")
    cj = lambda j: f"%{O['c'] + j}"
    r = lambda k: f"%{O['r'] + k}"
    C, c0, c1 = "v[2:3]", "v2", "v3"
    D, d0, d1 = "v[4:5]", "v4", "v5"
    lo = lambda k: "v2" if k == 9 else f"v{6 + 2 * (k - 10)}"
    hi = lambda k: "v3" if k == 9 else f"v{7 + 2 * (k - 10)}"
    K31264, K256, K977, SD = f"%{O['k31264']}", f"%{O['k256']}", f"%{O['k977']}", f"%{O['sd']}"
    K8192 = f"%{O['k8192']}"  # VOP3 takes no literal on gfx950: 2^13 from an SGPR
    L = []
    for k in range(17):
        if k <= 9:
            acc, first = C, True
            if k > 0:
                L.append(f"v_lshrrev_b64 {C}, 29, {C}")
                first = False
        else:
            acc = PAIR2[k]
            L.append(f"v_mad_u64_u32 {acc}, {SD}, {hi(k - 1)}, 8, 0")  # 8 * floor(C_{k-1} / 2^32)
            first = False
        for (x, y) in terms_of_column(k):
            L.append(f"v_mad_u64_u32 {acc}, {SD}, {opnd(x)}, {opnd(y)}, {'0' if first else acc}")
            first = False
        if k <= 8:
            L.append(f"v_and_b32_e32 {r(k)}, 0x1fffffff, {c0}")
    L.append(f"v_lshlrev_b32 {c1}, 3, {hi(16)}")          # o17 = 8 hi(P_16) (C's high word is free)
    # limbs 0..7: c = o_j + carry + 31264 o_{j+9} + 256 o_{j+8}
    L.append(f"v_mov_b32 {d1}, 0")
    if addend:
        L.append(f"v_add_u32 {d0}, {r(0)}, {cj(0)}")
    else:
        L.append(f"v_mov_b32 {d0}, {r(0)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(9)}, {K31264}, {D}")
    L.append(f"v_and_b32_e32 {r(0)}, 0x1fffffff, {d0}")
    for j in range(1, 8):
        L.append(f"v_lshrrev_b64 {D}, 29, {D}")           # carry < 2^19: the high word is 0
        if addend:
            L.append(f"v_add3_u32 {d0}, {d0}, {r(j)}, {cj(j)}")
        else:
            L.append(f"v_add_u32 {d0}, {d0}, {r(j)}")
        L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(j + 9)}, {K31264}, {D}")
        L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(j + 8)}, {K256}, {D}")
        L.append(f"v_and_b32_e32 {r(j)}, 0x1fffffff, {d0}")
    # limb 8: o_8 + carry + 31264 o17 + 256 o_16; 24 bits stay, the rest (units of 2^256) is T
    L.append(f"v_lshrrev_b64 {D}, 29, {D}")
    if addend:
        L.append(f"v_add3_u32 {d0}, {d0}, {r(8)}, {cj(8)}")
    else:
        L.append(f"v_add_u32 {d0}, {d0}, {r(8)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {c1}, {K31264}, {D}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(16)}, {K256}, {D}")
    L.append(f"v_and_b32_e32 {r(8)}, 0xffffff, {d0}")
    L.append(f"v_lshrrev_b64 {D}, 24, {D}")
    T, t0, t1 = "v[6:7]", "v6", "v7"                      # P_10 is dead by now
    L.append(f"v_mad_u64_u32 {T}, {SD}, {c1}, {K8192}, {D}")  # T = (c >> 24) + o17 2^13 < 2^37
    # 2^256 == 2^32 + 977: limb 0 += 977 T, limb 1 += 8 T (+ carries), limb 2 += carry
    L.append(f"v_mov_b32 {d1}, 0")
    L.append(f"v_mov_b32 {d0}, {r(0)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {t0}, {K977}, {D}")
    L.append(f"v_mad_u32_u24 {d1}, {t1}, {K977}, {d1}")
    L.append(f"v_and_b32_e32 {r(0)}, 0x1fffffff, {d0}")
    L.append(f"v_lshrrev_b64 {D}, 29, {D}")
    L.append(f"v_lshl_add_u64 {D}, {T}, 3, {D}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {r(1)}, 1, {D}")
    L.append(f"v_and_b32_e32 {r(1)}, 0x1fffffff, {d0}")
    L.append(f"v_alignbit_b32 {t0}, {d1}, {d0}, 29")
    L.append(f"v_add_u32 {r(2)}, {r(2)}, {t0}")
    return L


# ---------------------------------------------------------------------------- column form 3
# 1: the high columns emitted round-robin across their independent chains (measured equal at two
# waves per SIMD, profiles/r04/ab/il_*.json: the other wave already hides the chains' latency)
INTERLEAVE3 = os.environ.get("GSV_FE9_INTERLEAVE", "0") == "1"

def full_lines3(terms_of_column, addend=False):
    """Form 3: form 2's high columns, computed FIRST (column 9 from 0 instead of column 8's carry),
    and the low columns 0..8 never carried on their own: limb j's running value is the reduction's
    carry + column j's products + 31264 o_{j+9} + 256 o_{j+8} (+ c_j), one 64-bit multiply-add chain,
    then one mask and one 64-bit shift.  Form 2 carried every low column (shift + mask) and then ran
    the reduction's own carry chain over the masked limbs (a 32-bit add, a mask and a shift again):
    per product 9 64-bit shifts, 9 masks and 9 adds fewer.  Bounds: a column's products sum to
    < 63 2^58 (the m_a m_b <= 7 precondition), the carry is < 2^35, the folds < 2^47 + 2^40 and the
    addend < 2^31: < 2^64.  Limb 8's remainder c >> 24 < 2^40 and o17 < 2^32 make T < 2^46.  With an
    addend, c_j enters as one multiply-add by 1 (the three-operand add of form 2 is gone with the
    separate column carry)."""
    O = OPND2
    opnd = lambda x: f"%{O['a'] + x}" if x < 9 else (f"%{O['b'] + x - 9}" if x < 18 else f"%{O['c'] + x - 18}")
    cj = lambda j: f"%{O['c'] + j}"
    r = lambda k: f"%{O['r'] + k}"
    C, c0, c1 = "v[2:3]", "v2", "v3"
    D, d0, d1 = "v[4:5]", "v4", "v5"
    lo = lambda k: "v2" if k == 9 else f"v{6 + 2 * (k - 10)}"
    hi = lambda k: "v3" if k == 9 else f"v{7 + 2 * (k - 10)}"
    K31264, K256, K977, SD = f"%{O['k31264']}", f"%{O['k256']}", f"%{O['k977']}", f"%{O['sd']}"
    K8192 = f"%{O['k8192']}"
    L = []
    acc_of = lambda k: C if k == 9 else PAIR2[k]
    if INTERLEAVE3:
        # the eight high columns' product chains are independent: emitted round-robin (one term of
        # each column in turn), each from 0; the carries 8 hi(P_{k-1}) follow as one short chain
        cols = {k: list(terms_of_column(k)) for k in range(9, 17)}
        for t in range(max(len(v) for v in cols.values())):
            for k in range(9, 17):
                if t < len(cols[k]):
                    x, y = cols[k][t]
                    acc = acc_of(k)
                    L.append(f"v_mad_u64_u32 {acc}, {SD}, {opnd(x)}, {opnd(y)}, {'0' if t == 0 else acc}")
        for k in range(10, 17):
            acc = acc_of(k)
            L.append(f"v_mad_u64_u32 {acc}, {SD}, {hi(k - 1)}, 8, {acc if cols[k] else '0'}")
    else:
        for k in range(9, 17):                             # high columns: form 2's chains
            if k == 9:
                acc, first = C, True
            else:
                acc = PAIR2[k]
                L.append(f"v_mad_u64_u32 {acc}, {SD}, {hi(k - 1)}, 8, 0")
                first = False
            for (x, y) in terms_of_column(k):
                L.append(f"v_mad_u64_u32 {acc}, {SD}, {opnd(x)}, {opnd(y)}, {'0' if first else acc}")
                first = False
    L.append(f"v_lshlrev_b32 {c1}, 3, {hi(16)}")           # o17 = 8 hi(P_16) < 2^32
    for j in range(9):                                     # low limbs: products + folds, one carry
        first = j == 0
        if addend:
            L.append(f"v_mad_u64_u32 {D}, {SD}, {cj(j)}, 1, {'0' if first else D}")
            first = False
        for (x, y) in terms_of_column(j):
            L.append(f"v_mad_u64_u32 {D}, {SD}, {opnd(x)}, {opnd(y)}, {'0' if first else D}")
            first = False
        if j < 8:
            L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(j + 9)}, {K31264}, {D}")
            if j:
                L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(j + 8)}, {K256}, {D}")
            L.append(f"v_and_b32_e32 {r(j)}, 0x1fffffff, {d0}")
            L.append(f"v_lshrrev_b64 {D}, 29, {D}")       # carry < 2^35
        else:
            L.append(f"v_mad_u64_u32 {D}, {SD}, {c1}, {K31264}, {D}")
            L.append(f"v_mad_u64_u32 {D}, {SD}, {lo(16)}, {K256}, {D}")
            L.append(f"v_and_b32_e32 {r(8)}, 0xffffff, {d0}")
            L.append(f"v_lshrrev_b64 {D}, 24, {D}")
    T, t0, t1 = "v[6:7]", "v6", "v7"                      # P_10 is dead by now
    L.append(f"v_mad_u64_u32 {T}, {SD}, {c1}, {K8192}, {D}")  # T = (c >> 24) + o17 2^13 < 2^46
    L.append(f"v_mov_b32 {d1}, 0")
    L.append(f"v_mov_b32 {d0}, {r(0)}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {t0}, {K977}, {D}")
    L.append(f"v_mad_u32_u24 {d1}, {t1}, {K977}, {d1}")
    L.append(f"v_and_b32_e32 {r(0)}, 0x1fffffff, {d0}")
    L.append(f"v_lshrrev_b64 {D}, 29, {D}")
    L.append(f"v_lshl_add_u64 {D}, {T}, 3, {D}")
    L.append(f"v_mad_u64_u32 {D}, {SD}, {r(1)}, 1, {D}")
    L.append(f"v_and_b32_e32 {r(1)}, 0x1fffffff, {d0}")
    L.append(f"v_alignbit_b32 {t0}, {d1}, {d0}, 29")
    L.append(f"v_add_u32 {r(2)}, {r(2)}, {t0}")
    return L


def full2(name, doc, terms_of_column, addend=False, dot=False, gen=None):
    L = (gen or full_lines2)(terms_of_column, addend)
    outs = ", ".join([f'"=&v"(r[{i}])' for i in range(9)] + ['"=&s"(sd)'])
    ins = ", ".join([f'"v"(a[{i}])' for i in range(9)] + [f'"v"(b[{j}])' for j in range(9)] +
                    ['"s"(k31264)', '"s"(k256)', '"s"(k977)', '"s"(k8192)'] +
                    ([f'"v"(c[{j}])' for j in range(9)] if addend or dot else []) +
                    ([f'"v"(d[{j}])' for j in range(9)] if dot else []))
    body = "\\n\\t".join(L)
    clob = ", ".join(f'"v{i}"' for i in range(2, 20))
    return [f"// {doc}",
            f"__device__ __forceinline__ void {name}(uint32_t r[9], const uint32_t a[9], const uint32_t b[9]"
            + (", const uint32_t c[9]" if addend or dot else "") + (", const uint32_t d[9]" if dot else "") + ") {",
            "    uint64_t sd;",
            "    uint32_t k31264 = 31264u, k256 = 256u, k977 = 977u, k8192 = 8192u;",
            f'    asm("{body}"',
            f"        : {outs}",
            f"        : {ins}",
            f"        : {clob});",
            "}"]

def main():
    out = ["// GENERATED by tools/gen_fe9_asm.py — do not edit by hand.",
           "// Column products of secp256k1_fe9.cuh as single inline-asm statements (see the generator's",
           "// docstring for why).  Column form 3: the low columns run inside the reduction's carry chain",
           "// (full_lines3).  Forms 1 (every column masked and shifted) and 2 (high columns 9..16 unmasked in",
           "// fixed register pairs) stay in the generator as the instruction emulator's references",
           "// (tests/test_asm_emulated.py); the kernels use form 3 only (r04: 175 -> 136 instructions a product).",
           "#pragma once", "#include <stdint.h>",
           "namespace gsv {"]
    specs = [("fe9_mul_full", "r = a * b mod p, weakly normalised (fe9_mul's contract)", MUL_TERMS, False, False),
             ("fe9_sqr_full", "r = a^2 mod p with b = 2a limb-wise (fe9_sqr's contract)", SQR_TERMS, False, False),
             ("fe9_mul_add_full", "r = a * b + c mod p, c limbs < 2^31 (fe9_mul_add's contract)", MUL_TERMS, True, False),
             ("fe9_sqr_add_full", "r = a^2 + c mod p with b = 2a limb-wise, c limbs < 2^31 (fe9_sqr_add's contract)",
              SQR_TERMS, True, False),
             ("fe9_dot_full", "r = a * b + c * d mod p, one reduction (fe9_dot's contract)", DOT_TERMS, False, True)]
    for name, doc, terms, add, dot in specs:
        out += full2(name, doc, terms, add, dot, gen=full_lines3)
    out.append("}  // namespace gsv")
    with open(OUT, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
