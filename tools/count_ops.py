"""Operation counts of OUR kernels per unit of work, from the instrumented build
(geth-sharding_amd/csrc/opcount.cuh; built by `VSRCS="ecrecover bn256 notary collation"
tools/build_variant.sh opcount -DGSV_OPCOUNT`), at the bench's batch sizes:

    recovery       one k_ecrecover lane of the configs[1] batch (2^20 signatures)
    pairing_check  one 4-pair check of the configs[4] batch on one GPU (65,536 checks) and of the
                   per-rank batch at N = 8 (8,192 checks: another lane layout, §3.4 of DESIGN.md)

"mac_equiv" weights every 256-bit product the way SURVEY.md §8d weights the reference's: a
product = 8 x 8 = 64 32x32-bit partial products, a squaring 36, a BN254 Montgomery product 64 + 64
= 128.  Safegcd inversions (ours) are counted separately: they replace the reference's
exponentiation-based inversions, whose products the reference figure includes.

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

KINDS = ["fe_mul", "fe_sqr", "sc_mul", "sc_sqr", "bn_mul", "modinv"]


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
    out = {"build": "variants/opcount (-DGSV_OPCOUNT)", "weights": {"fe_mul": 64, "fe_sqr": 36, "sc_mul": 64,
                                                                      "sc_sqr": 36, "bn_mul": 128}}
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
    c["mac_equiv"] = round(64 * c.get("fe_mul", 0) + 36 * c.get("fe_sqr", 0) + 64 * c.get("sc_mul", 0)
                           + 36 * c.get("sc_sqr", 0), 1)
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
        c["mac_equiv"] = round(128 * c.get("bn_mul", 0), 1)
        out[name] = c
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
