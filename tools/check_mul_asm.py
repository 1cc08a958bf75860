"""CPU emulation of the generated single-statement products in mul_asm.cuh (mul_8x8_fx,
sqr_8_fx): interprets the asm text for the VALU subset they use and checks the products
against Python integers on random and edge-case limbs.  Run after tools/gen_mul_asm.py."""
import os
import random
import re
import sys

M32 = (1 << 32) - 1
SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "geth-sharding_amd", "csrc", "mul_asm.cuh")


def functions(text):
    out = {}
    for m in re.finditer(r"void (\w+_fx)\(([^)]*)\) \{\n(.*?)\n\}", text, re.S):
        name, body = m.group(1), m.group(3)
        asm = re.search(r'asm volatile\("(.*?)" : (.*?) : (.*?) : ', body, re.S)
        ins = asm.group(1).split("\\n\\t")
        outs = re.findall(r'"=&?[vs]"\((\w+)(?:\[(\d+)\])?\)', asm.group(2))
        inps = re.findall(r'"[vs]"\((\w+)\[(\d+)\]\)', asm.group(3))
        out[name] = (ins, outs, inps)
    return out


def run(prog, env):
    """env: operand index -> value (32-bit or 64-bit for the SGPR dummy), plus fixed regs."""
    regs = {}

    def rd(tok):
        tok = tok.strip()
        if tok.startswith("%"):
            return env[int(tok[1:])]
        if tok.startswith("v["):
            a, b = map(int, re.findall(r"\d+", tok))
            return regs.get(f"v{a}", 0) | (regs.get(f"v{b}", 0) << 32)
        if tok == "vcc":
            return regs.get("vcc", 0)
        if re.fullmatch(r"v\d+", tok):
            return regs[tok]
        return int(tok, 0)

    def wr(tok, val, width=32):
        tok = tok.strip()
        if tok.startswith("%"):
            env[int(tok[1:])] = val & ((1 << width) - 1)
        elif tok.startswith("v["):
            a, b = map(int, re.findall(r"\d+", tok))
            regs[f"v{a}"] = val & M32
            regs[f"v{b}"] = (val >> 32) & M32
        else:
            regs[tok] = val & ((1 << width) - 1)

    for line in prog:
        op, rest = line.split(None, 1)
        a = [x.strip() for x in rest.split(",")]
        if op == "v_mad_u64_u32":
            r = rd(a[2]) * rd(a[3]) + rd(a[4])
            wr(a[0], r, 64)
            wr(a[1], r >> 64, 64)
        elif op in ("v_addc_co_u32_e64", "v_addc_co_u32_e32"):
            r = rd(a[2]) + rd(a[3]) + (rd(a[4]) & 1)
            wr(a[0], r)
            wr(a[1], r >> 32, 64)
        elif op in ("v_add_co_u32_e64", "v_add_co_u32_e32"):
            r = rd(a[2]) + rd(a[3])
            wr(a[0], r)
            wr(a[1], r >> 32, 64)
        elif op == "v_mov_b32":
            wr(a[0], rd(a[1]))
        else:
            raise SystemExit(f"unhandled {op}")
    return env


def limbs(x, n):
    return [(x >> (32 * i)) & M32 for i in range(n)]


def main():
    fns = functions(open(SRC).read())
    rng = random.Random(1)
    edge = [0, 1, M32, (1 << 256) - 1, (1 << 256) - (1 << 32) - 977, 1 << 255, (1 << 224) - 1]
    vals = edge + [rng.getrandbits(256) for _ in range(2000)] + [rng.getrandbits(256) | (((1 << 128) - 1) << 128) for _ in range(200)]
    nfail = 0
    for name, (prog, outs, inps) in fns.items():
        nout = len(outs)
        for idx, x in enumerate(vals):
            y = vals[(idx * 7 + 3) % len(vals)]
            env = {}
            av, bv = limbs(x, 8), limbs(y, 8)
            for k, (arr, i) in enumerate(inps):
                env[nout + k] = (av if arr == "a" else bv)[int(i)]
            env = run(prog, env)
            got = sum(env[k] << (32 * k) for k in range(nout) if outs[k][0] == "t")
            na = sum(1 for arr, _ in inps if arr == "a")
            nb = sum(1 for arr, _ in inps if arr == "b")
            xa, yb = x & ((1 << (32 * na)) - 1), y & ((1 << (32 * nb)) - 1)
            want = xa * xa if name.startswith("sqr") else xa * yb
            if got != want:
                nfail += 1
                if nfail < 5:
                    print(name, hex(x), hex(y), "MISMATCH")
        print(f"{name}: {len(prog)} instructions, {sum(1 for l in prog if l.startswith('v_mad'))} v_mad_u64_u32, {len(vals)} cases")
    if nfail:
        sys.exit(f"{nfail} mismatches")
    print("all products exact")


if __name__ == "__main__":
    main()
