"""Operation counts of OUR kernels per unit of work, from the instrumented build
(geth-sharding_amd/csrc/opcount.cuh; built by `VSRCS="ecrecover bn256 notary collation"
tools/build_variant.sh opcount -DGSV_OPCOUNT`), at the bench's batch sizes:

    recovery       one k_ecrecover lane of the configs[1] batch (2^20 signatures)
    pairing_check  one 4-pair check of the configs[4] batch on one GPU (65,536 checks) and of the
                   per-rank batch at N = 8 (8,192 checks: another lane layout, §3.4 of DESIGN.md)
    notary_tx      one transaction of the configs[3] step (100 shards x 8,192 txs through k_notary_tx:
                   RLP decode, sighash, recovery, address; every 128th tx invalid by construction)

"mad" is the number of v_mad_u64_u32 (32 x 32 -> 64-bit multiply-adds: the unit of the VALU MAC
roofline) our kernels execute, from the op counts and each op's mad count in our limb layout:
a secp256k1 fe9 product 81 + 27 (column form 3 of tools/gen_fe9_asm.py: 7 high-column carries, 17
2^261 folds, 3 in the 2^256 fold; a product with an addend has 9 more, counted as a product), a
squaring 45 + 27, a dot product 162 + 27,
a scalar product 64 (8 x 32-bit limbs; the folds mod n are not counted, < 1 %), a BN254 F_p product
81 (9 x 29-bit) and a BN254 Montgomery reduction 81 (one per fq_mul / fq_mul2 / fq_dot, shared by
the products it sums).  Safegcd inversions are counted separately (their divsteps are not mads).
"mac_equiv" is the same count (kept under the name the bench reads).

    python tools/count_ops.py > profiles/r02/opcount.json        (on the GPU box)
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GSV_LIB_PATH"] = os.path.join(ROOT, "variants", "opcount", "libgsv.so")
sys.path.insert(0, os.path.join(ROOT, "geth-sharding_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import gsv  # noqa: E402
from gsv import _lib  # noqa: E402

KINDS = ["fe_mul", "fe_sqr", "sc_mul", "sc_sqr", "bn_mul", "modinv", "bn_redc", "fe_dot"]


def read(tu):
    buf = (ctypes.c_ulonglong * 8)()
    rc = getattr(_lib.load(), f"gsv_opcount_{tu}")(buf, 1)
    assert rc == 0, f"gsv_opcount_{tu} failed (is {os.environ['GSV_LIB_PATH']} the -DGSV_OPCOUNT build?)"
    return dict(zip(KINDS, list(buf)[:len(KINDS)]))


def per_unit(c, n):
    return {k: round(v / n, 3) for k, v in c.items() if v}


def main():
    ctx = gsv.Context(0)
    dev = torch.device("cuda", 0)
    W = {"fe_mul": 108, "fe_sqr": 72, "sc_mul": 64, "sc_sqr": 36, "bn_mul": 81, "bn_redc": 81, "fe_dot": 189}
    out = {"build": "variants/opcount (-DGSV_OPCOUNT)", "unit": "v_mad_u64_u32 per unit of work",
           "weights_mad_per_op": W}
    # ---- configs[1]: 2^20 recoveries
    n = 1 << 20
    msg = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    pub = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    st = torch.empty((n,), dtype=torch.uint8, device=dev)
    ctx.synth_sign_dev(1000, msg, sig)
    torch.cuda.synchronize()
    read("ecrecover")  # drop the signer's counts
    ctx.ecrecover_batch_dev(msg, sig, pub, addr, st)
    torch.cuda.synchronize()
    assert int(st.max()) == 0
    c = per_unit(read("ecrecover"), n)
    c["mac_equiv"] = round(sum(W[k] * c.get(k, 0) for k in ("fe_mul", "fe_sqr", "sc_mul", "sc_sqr", "fe_dot")), 1)
    out["recovery"] = c
    # ---- configs[4]: 4-pair checks, one GPU's batch and the 8-rank per-rank batch
    for name, nchk in (("pairing_check", 65536), ("pairing_check_8192", 8192)):
        pin = torch.empty((nchk, 768), dtype=torch.uint8, device=dev)
        pexp = torch.empty((nchk,), dtype=torch.uint8, device=dev)
        pver = torch.empty((nchk,), dtype=torch.uint8, device=dev)
        ctx.bn256_synth_checks_dev(5000, pin, pexp)
        off = np.arange(nchk + 1, dtype=np.uint64) * 768
        ctx.pairing_prepare(off)
        torch.cuda.synchronize()
        read("bn256")  # drop the generator's counts
        ctx.pairing_check_batch_dev(pin, off, pver, prepare=False)
        torch.cuda.synchronize()
        assert torch.equal(pver, pexp)
        c = per_unit(read("bn256"), nchk)
        c["fp_products"] = c.get("bn_mul", 0)
        c["mac_equiv"] = round(W["bn_mul"] * c.get("bn_mul", 0) + W["bn_redc"] * c.get("bn_redc", 0), 1)
        out[name] = c
    # ---- configs[3]: the notary step's transactions
    nsh, txs = 100, 8192
    bodies = torch.empty((nsh * txs * 128,), dtype=torch.uint8, device=dev)
    exp = torch.empty((nsh * txs,), dtype=torch.uint8, device=dev)
    ctx.notary_synth_dev(777, 0, nsh, txs, bodies, exp)
    noff = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    ctx.notary_prepare(noff, max_txs=txs)
    torch.cuda.synchronize()
    read("notary")  # drop the generator's counts
    r = torch.empty((nsh, 32), dtype=torch.uint8, device=dev)
    cnt = torch.empty((nsh,), dtype=torch.int32, device=dev)
    bm = torch.empty((nsh, txs // 8), dtype=torch.uint8, device=dev)
    stt = torch.empty((nsh, txs), dtype=torch.uint8, device=dev)
    ctx.notary_validate_shards_dev(bodies, noff, r, cnt, bm, None, stt, max_txs=txs, prepare=False)
    torch.cuda.synchronize()
    assert torch.equal(stt.view(-1), exp)
    c = per_unit(read("notary"), nsh * txs)
    c["mac_equiv"] = round(sum(W[k] * c.get(k, 0) for k in ("fe_mul", "fe_sqr", "sc_mul", "sc_sqr", "fe_dot")), 1)
    out["notary_tx"] = c
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
