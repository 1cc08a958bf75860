"""CPU checks of the full-size config fixtures (tests/golden/configs.json) against the oracle and,
where it is built, the reference's own C code: the generators and the restatement reproduce the
committed values on samples, so the GPU tests in test_gpu_configs.py compare against pinned data."""
import ctypes
import hashlib
import os
import struct
import sys

import numpy as np
import pytest

from conftest import golden

HERE = os.path.dirname(os.path.abspath(__file__))
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def test_configs0_sender_on_cpu(oracle):
    if oracle.ref() is None:
        pytest.skip("oracle/_ref not built")
    from oracle import cfg0
    g = golden("configs.json")["configs0_sender"]
    txs, addrs = cfg0.eip155_txs(g["n"])
    assert hashlib.sha256(b"".join(txs)).hexdigest() == g["txs_sha256"]
    assert hashlib.sha256(addrs.tobytes()).hexdigest() == g["senders_sha256"]
    flat = np.frombuffer(b"".join(txs) + b"\0", np.uint8)
    off = np.zeros(len(txs) + 1, np.uint64)
    off[1:] = np.cumsum([len(t) for t in txs])
    assert cfg0.use_reference_crypto() == "reference"
    try:
        a, st, _ = cfg0.sender_many(flat, off, len(txs), 8)
    finally:
        oracle.lib().oracle_set_crypto(None, None)
    assert (st == 0).all() and hashlib.sha256(a.tobytes()).hexdigest() == g["senders_sha256"]
    # the restatement's own crypto agrees on a sample
    a2, st2, _ = cfg0.sender_many(flat, off[:257], 256, 4)
    assert (st2 == 0).all() and (a2 == addrs[:256]).all()


def test_configs1_rows_match_restated_signer(oracle):
    g = golden("configs.json")["configs1_ecrecover"]
    for i, row in enumerate(g["first"]):
        def der(tag):
            return oracle.keccak256(struct.pack("<QQ", g["seed"], i) + tag)
        d = (int.from_bytes(der(b"key"), "big") % N_ORDER or 1).to_bytes(32, "big")
        k = (int.from_bytes(der(b"nce"), "big") % N_ORDER or 1).to_bytes(32, "big")
        assert row["msg"] == der(b"msg").hex()
        assert row["sig"] == oracle.secp_sign(der(b"msg"), d, k).hex()
        rc, pub = oracle.ecrecover(bytes.fromhex(row["msg"]), bytes.fromhex(row["sig"]))
        assert rc == 1 and pub.hex() == row["pub"] == oracle.secp_pubkey(d).hex()
        assert row["addr"] == oracle.keccak256(pub[1:])[12:].hex()


def test_configs2_first_root(oracle):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import xoshiro_bytes
    g = golden("configs.json")["configs2_chunk_roots"]
    assert len(g["roots"]) == 100 and len(set(g["roots"])) == 100
    assert oracle.derive_sha_bytes(xoshiro_bytes(g["seeds"][7], g["n"])).hex() == g["roots"][7]


def test_configs4_sample_verdicts(oracle):
    """The committed configs[4] verdicts follow the generator's classes (make_golden.configs4_inputs),
    and a sample of checks rebuilt on the CPU gets the committed verdict from the oracle."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import configs4_inputs
    g = golden("configs.json")["configs4_pairing"]
    v = g["verdicts"]
    assert g["n"] == 65536 and len(v) == g["first"] == 1024
    bad = {300, 400, 500, 1023}
    assert all(v[i] == ("2" if i in bad else "0" if i % 8 == 7 else "1") for i in range(1024))
    per = g["n"] // 1024
    assert g["verdict_counts"] == {"0": per * 127, "1": per * 893, "2": per * 4}  # 1023 is bad, not false
    for c in (0, 7, 100, 200, 300, 400, 500, 1023, 1024 + 300, 65535):
        r = oracle.pairing_check(configs4_inputs(c, g["seed"]))
        want = 2 if c % 1024 in bad else 0 if c % 8 == 7 else 1
        assert (2 if r < 0 else r) == want, c
