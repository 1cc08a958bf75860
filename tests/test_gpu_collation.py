"""GPU parity for SURVEY.md §8f rows 2-3: DeriveSha over arbitrary lists (tx / receipt roots),
Proof of Custody (Collation.CalculatePOC) and collation header hash + proposer signature, through the
C ABI, against the committed fixtures (tests/golden/collation.json, oracle-generated and pinned by
tests/test_oracle.py) and the live oracle."""
import os
import random
import sys

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _xoshiro(seed, n):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_golden import xoshiro_bytes
    return xoshiro_bytes(seed, n)


def test_derive_sha_fixtures(ctx):
    g = golden("collation.json")["derive_sha"] + golden("trie.json")["derive_sha"]
    lists = [[bytes.fromhex(x) for x in c["items"]] for c in g]
    lists.append([])
    want = [c["root"] for c in g] + [golden("trie.json")["empty_root"]]
    out = ctx.derive_sha_batch(lists)
    for i, w in enumerate(want):
        assert bytes(out[i]).hex() == w, (i, len(lists[i]))


def test_derive_sha_random_vs_oracle(ctx, oracle):
    # ragged batch of lists with mixed lengths (several lists share N: one plan, one launch set)
    rng = random.Random(21)
    lists = []
    for n in [0, 1, 1, 2, 5, 15, 16, 16, 17, 31, 32, 33, 100, 128, 129, 255, 256, 257, 513, 4097, 300, 1]:
        lists.append([bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 1, 3, 31, 32, 60, 140, 700])))
                      for _ in range(n)])
    out = ctx.derive_sha_batch(lists)
    for i, lst in enumerate(lists):
        assert bytes(out[i]) == oracle.derive_sha(lst), (i, len(lst))


def test_derive_sha_byte_lists_equal_chunk_root(ctx):
    # Chunks(body).GetRlp(j) as explicit items == the specialised chunk-root kernels
    rng = np.random.default_rng(3)
    bodies = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in [1, 17, 256, 4096, 70000]]
    lists = [[b"\x80" if b == 0 else bytes([b]) if b < 128 else bytes([0x81, b]) for b in body] for body in bodies]
    a = ctx.derive_sha_batch(lists)
    b = ctx.chunk_root_batch(bodies)
    assert (a == b).all()


def test_derive_sha_dev(ctx, oracle):
    import torch
    rng = random.Random(4)
    lists = [[bytes(rng.getrandbits(8) for _ in range(rng.randint(1, 200))) for _ in range(n)] for n in [3, 50, 50]]
    items = [x for lst in lists for x in lst]
    voff = np.zeros(len(items) + 1, np.uint64)
    voff[1:] = np.cumsum([len(x) for x in items])
    list_off = np.array([0, 3, 53, 103], np.uint64)
    vals = torch.tensor(list(b"".join(items)), dtype=torch.uint8, device="cuda")
    roots = torch.zeros((3, 32), dtype=torch.uint8, device="cuda")
    ctx.derive_sha_batch_dev(vals, voff, list_off, roots)
    torch.cuda.synchronize()
    r = roots.cpu().numpy()
    for i, lst in enumerate(lists):
        assert bytes(r[i]) == oracle.derive_sha(lst)


def test_poc_fixtures(ctx):
    for c in golden("collation.json")["poc"]:
        body = bytes.fromhex(c["body"]) if c["body"] is not None else _xoshiro(c["xoshiro_seed"], c["n"])
        out = ctx.collation_poc_batch([body], bytes.fromhex(c["salt"]))
        assert bytes(out[0]).hex() == c["poc"], (len(body), len(c["salt"]) // 2)


def test_poc_batch_vs_oracle(ctx, oracle):
    rng = np.random.default_rng(9)
    salt = bytes(range(7, 27))  # 20-byte salt (sharding/collation_test.go:318)
    bodies = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in [0, 1, 2, 300, 300, 5000]]
    out = ctx.collation_poc_batch(bodies, salt)
    for i, b in enumerate(bodies):
        assert bytes(out[i]) == oracle.calculate_poc(b, salt), i


@pytest.mark.parametrize("slen", [0, 1, 3, 15, 16, 17, 20, 33, 255, 9000])
def test_poc_salt_lengths_vs_oracle(ctx, oracle, slen):
    """k_poc_expand writes 16 salted bytes per thread from the period-(s+1) pattern staged in LDS plus
    the window's body bytes (one or more per window below s = 15, at most one from s = 15 up; every
    window phase); salts past its LDS bound (8,192 bytes) take k_poc_expand_bytes.  Bodies of 0-1,037
    bytes, so salted lengths end at every phase of a 16-byte store."""
    rng = np.random.default_rng(100 + slen)
    salt = rng.integers(0, 256, slen, dtype=np.uint8).tobytes()
    lens = [0, 1, 2, 15, 16, 17, 100, 1037] if slen < 9000 else [0, 1, 7, 100]
    bodies = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    out = ctx.collation_poc_batch(bodies, salt)
    for i, b in enumerate(bodies):
        assert bytes(out[i]) == oracle.calculate_poc(b, salt), (slen, len(b))


def test_poc_size_limit(ctx):
    import gsv
    with pytest.raises(gsv.GsvError):
        ctx.collation_poc_batch([bytes(1 << 20)], bytes(64))  # 65 MiB salted body > 2^26


def _headers(cases):
    n = len(cases)
    sid = np.zeros((n, 32), np.uint8)
    per = np.zeros((n, 32), np.uint8)
    root = np.zeros((n, 32), np.uint8)
    prop = np.zeros((n, 20), np.uint8)
    sig = np.zeros((n, 65), np.uint8)
    nil = np.zeros(n, np.uint8)
    for i, c in enumerate(cases):
        sid[i] = np.frombuffer(int(c["shard_id"]).to_bytes(32, "big"), np.uint8)
        per[i] = np.frombuffer(int(c["period"]).to_bytes(32, "big"), np.uint8)
        if c["chunk_root"] is None:
            nil[i] |= 1
        else:
            root[i] = np.frombuffer(bytes.fromhex(c["chunk_root"]), np.uint8)
        if c["proposer"] is None:
            nil[i] |= 2
        else:
            prop[i] = np.frombuffer(bytes.fromhex(c["proposer"]), np.uint8)
        if not c["sig"]:
            nil[i] |= 4
        else:
            sig[i] = np.frombuffer(bytes.fromhex(c["sig"]), np.uint8)
    return sid, root, per, prop, sig, nil


def test_header_hash_kat(ctx):
    kat = golden("collation.json")["header_kat"]
    h, _, _ = ctx.collation_header_verify_batch(*_headers(kat))
    for i, c in enumerate(kat):
        assert bytes(h[i]).hex() == c["hash"], c["note"]


def test_header_proposer_signatures(ctx):
    import gsv
    cases = golden("collation.json")["signed_headers"]
    h, signer, st = ctx.collation_header_verify_batch(*_headers(cases))
    want = {"ok": gsv._lib.ST_OK, "mismatch": gsv._lib.ST_PROPOSER_MISMATCH,
            "invalid_recid": gsv._lib.ST_INVALID_RECID, "recover_failed": gsv._lib.ST_RECOVER_FAILED}
    for i, c in enumerate(cases):
        assert bytes(h[i]).hex() == c["hash"], i
        assert st[i] == want[c["expect"]], (i, c["expect"], st[i])
        if c["expect"] in ("ok", "mismatch"):
            assert bytes(signer[i]).hex() == c["signer"], i
        else:
            assert not signer[i].any()


def test_sharding_mirror_api(ctx, oracle):
    from gsv import sharding as S
    c = golden("collation.json")["signed_headers"][0]
    hdr = S.CollationHeader(c["shard_id"], bytes.fromhex(c["chunk_root"]), c["period"], bytes.fromhex(c["proposer"]))
    unsigned = hdr.Hash()
    assert unsigned == oracle.collation_header_hash(c["shard_id"], bytes.fromhex(c["chunk_root"]), c["period"],
                                                    bytes.fromhex(c["proposer"]), None)
    hdr.AddSig(bytes.fromhex(c["sig"]))
    assert hdr.Hash().hex() == c["hash"]
    signer, st = S.VerifyProposerSignatures([hdr])
    assert st[0] == 0 and bytes(signer[0]).hex() == c["signer"]
    col = S.Collation(S.CollationHeader(1, None, 1, None, b""), b"\x56\xff")
    col.CalculateChunkRoot()
    poc = col.CalculatePOC(b"\x01\x9f")
    assert poc != col.Header().ChunkRoot()
    assert poc.hex() == golden("collation.json")["poc"][0]["poc"]
    assert S.DeriveSha([bytes.fromhex(x) for x in golden("trie.json")["derive_sha"][0]["items"]]).hex() == \
        golden("trie.json")["derive_sha"][0]["root"]


def test_dev_calls_on_two_streams_share_the_workspace_safely(ctx, oracle):
    # *_dev calls return without a host sync; calls on different streams are ordered on the GPU
    # through the context's workspace event (gsv_api.hip work_begin/work_end)
    import torch
    rng = np.random.default_rng(17)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    sizes = [[70000, 3000, 129], [4096, 1 << 16], [17, 300000, 5, 1]]
    jobs = []
    for k, sz in enumerate(sizes):
        bodies = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sz]
        off = np.zeros(len(bodies) + 1, np.uint64)
        off[1:] = np.cumsum([len(b) for b in bodies])
        dev = torch.tensor(np.frombuffer(b"".join(bodies), np.uint8).copy(), device="cuda")
        roots = torch.zeros((len(bodies), 32), dtype=torch.uint8, device="cuda")
        st = s1 if k % 2 == 0 else s2
        st.wait_stream(torch.cuda.current_stream())  # the copy and zero fill run on the default stream
        ctx.chunk_root_batch_dev(dev, off, roots, stream=st)
        jobs.append((bodies, roots, dev))
    salt = bytes(range(3, 23))
    pb = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in [1000, 0, 64]]
    poff = np.zeros(4, np.uint64)
    poff[1:] = np.cumsum([len(b) for b in pb])
    pdev = torch.tensor(np.frombuffer(b"".join(pb) + b"\0", np.uint8).copy(), device="cuda")
    pocs = torch.zeros((3, 32), dtype=torch.uint8, device="cuda")
    s2.wait_stream(torch.cuda.current_stream())
    ctx.collation_poc_batch_dev(pdev, poff, salt, pocs, stream=s2)
    torch.cuda.synchronize()
    for bodies, roots, _ in jobs:
        r = roots.cpu().numpy()
        for i, b in enumerate(bodies):
            assert bytes(r[i]) == oracle.derive_sha_bytes(b), (len(b), i)
    p = pocs.cpu().numpy()
    for i, b in enumerate(pb):
        assert bytes(p[i]) == oracle.calculate_poc(b, salt), i


def test_derive_sha_dev_tx_lists_at_batch_edges(ctx, oracle):
    """k_derive_leaf reads a hashed leaf's value as whole 16-byte groups when every lane's value has
    >= 32 bytes of the batch on both sides, and dword by dword in the waves at the batch's edges.  Here
    the batch is a slice of the items (list_off starting past item 0, so bytes before it are other
    items') of 100-160-byte values (the tx-root leg's shape) plus short and empty values, in a vals
    buffer that ends at the last value with 0xff bytes after it."""
    import torch
    rng = np.random.default_rng(17)
    sizes = [5, 200, 64, 3, 200, 1]
    lists = [[rng.integers(0, 256, int(rng.choice([0, 1, 40, 100, 135, 150, 160])), dtype=np.uint8).tobytes()
              for _ in range(n)] for n in sizes]
    items = [x for lst in lists for x in lst]
    voff = np.zeros(len(items) + 1, np.uint64)
    voff[1:] = np.cumsum([len(x) for x in items])
    list_off = np.cumsum([0] + sizes).astype(np.uint64)
    flat = np.frombuffer(b"".join(items), np.uint8)
    vals = torch.full((len(flat) + 64,), 0xff, dtype=torch.uint8, device="cuda")
    vals[:len(flat)] = torch.from_numpy(flat.copy()).cuda()
    sub = list_off[1:]  # the batch: lists 1.. (item 0's list is outside it)
    roots = torch.zeros((len(sub) - 1, 32), dtype=torch.uint8, device="cuda")
    ctx.derive_sha_batch_dev(vals, voff, sub, roots)
    torch.cuda.synchronize()
    r = roots.cpu().numpy()
    for i, lst in enumerate(lists[1:]):
        assert bytes(r[i]) == oracle.derive_sha(lst), (i, len(lst))
