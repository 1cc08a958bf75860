"""GPU tests of the C-ABI contract itself: the ecrecover precompile entry point
(core/vm/contracts.go:78-101) against the oracle and the reference build, the *_dev prepare /
graph-capture promise of include/gsv.h, and the input validation the host entry points owe the
kernels."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


# ---------------------------------------------------------------- ecrecover precompile
def _precompile_oracle(oracle, inp: bytes):
    """contracts.go:78-101 restated over the oracle's recoverPlain (homestead = false)."""
    x = inp.ljust(128, b"\0")[:128]
    if any(x[32:63]):
        return None
    out = ctypes.create_string_buffer(20)
    st = oracle.lib().oracle_recover_plain(out, x[:32], x[64:96], 32, x[96:128], 32, x[63:64], 1, 0)
    return bytes(12) + out.raw if st == 0 else None


def test_precompile_reference_vector(ctx):
    # core/vm/contracts_test.go:390-398 (BenchmarkPrecompiledEcrecover)
    inp = bytes.fromhex(
        "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e"
        "000000000000000000000000000000000000000000000000000000000000001b"
        "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e"
        "789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02")
    from gsv.crypto import EcrecoverPrecompile
    out = EcrecoverPrecompile().Run(inp, ctx)
    assert out.hex() == "000000000000000000000000ceaccac640adf55b2028469bd36ba501f28b699d"
    assert EcrecoverPrecompile().RequiredGas(inp) == 3000


def test_precompile_edges_vs_oracle(ctx, oracle):
    rng = random.Random(78)
    inputs = []
    for i in range(400):
        key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
        m = bytes(rng.getrandbits(8) for _ in range(32))
        sig = oracle.secp_sign(m, key, rng.randrange(1, N_ORDER).to_bytes(32, "big"))
        r, s, v = sig[:32], sig[32:64], sig[64] + 27
        vword = bytearray(32)
        vword[31] = v
        kind = i % 16
        if kind == 1:      # input[32:63] not all zero -> nil
            vword[rng.randrange(0, 31)] = 1
        elif kind == 2:    # v = 29 / 26 / 0 / 255 -> invalid
            vword[31] = rng.choice([29, 26, 0, 255])
        elif kind == 3:    # high s: homestead=false accepts it (recovers another key)
            s = (N_ORDER - int.from_bytes(s, "big")).to_bytes(32, "big")
        elif kind == 4:    # r = 0
            r = bytes(32)
        elif kind == 5:    # s = n
            s = N_ORDER.to_bytes(32, "big")
        elif kind == 6:    # short input: right-padded (s and part of r become zero)
            inputs.append(m + bytes(vword) + r[:20])
            continue
        elif kind == 7:    # longer than 128 bytes: the tail is ignored
            inputs.append(m + bytes(vword) + r + s + b"\xff" * 40)
            continue
        elif kind == 8:    # empty input
            inputs.append(b"")
            continue
        elif kind == 9:    # r not an x-coordinate / random
            r = rng.randrange(1, N_ORDER).to_bytes(32, "big")
        inputs.append(m + bytes(vword) + r + s)
    out, ok = ctx.ecrecover_precompile_batch(inputs)
    for i, inp in enumerate(inputs):
        want = _precompile_oracle(oracle, inp)
        if want is None:
            assert ok[i] == 0 and not out[i].any(), i
        else:
            assert ok[i] == 1 and bytes(out[i]) == want, i
    assert ok.sum() > 150 and (ok == 0).sum() > 100


def test_precompile_matches_reference_build(ctx, oracle):
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref not built on this machine")
    rng = random.Random(79)
    inputs, want = [], []
    for _ in range(128):
        key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
        m = bytes(rng.getrandbits(8) for _ in range(32))
        sig = ctypes.create_string_buffer(65)
        R.gsvref_sign(sig, m, key)
        pub = ctypes.create_string_buffer(65)
        assert R.gsvref_pubkey(pub, key) == 1
        h = ctypes.create_string_buffer(32)
        R.gsvref_keccak256(h, pub.raw[1:], 64)
        inputs.append(m + bytes(31) + bytes([sig.raw[64] + 27]) + sig.raw[:64])
        want.append(bytes(12) + h.raw[12:])
    out, ok = ctx.ecrecover_precompile_batch(inputs)
    assert ok.all()
    assert [bytes(o) for o in out] == want


# ---------------------------------------------------------------- recoverPlain: V wider than 8 bits
def test_sender_batch_rejects_wide_v_without_flag(ctx, oracle):
    # v = 283 with v_big = 0: Vb.BitLen() > 8 -> ErrInvalidSig (transaction_signing.go:227)
    rng = random.Random(283)
    key = rng.randrange(1, N_ORDER).to_bytes(32, "big")
    m = bytes(rng.getrandbits(8) for _ in range(32))
    sig = oracle.secp_sign(m, key, rng.randrange(1, N_ORDER).to_bytes(32, "big"))
    H = np.frombuffer(m, np.uint8)[None].repeat(2, 0)
    R_ = np.frombuffer(sig[:32], np.uint8)[None].repeat(2, 0)
    S_ = np.frombuffer(sig[32:64], np.uint8)[None].repeat(2, 0)
    V = np.array([27 + sig[64] + 256, 27 + sig[64]], np.uint64)
    VB = np.zeros(2, np.uint8)
    addr, st = ctx.sender_batch(H, R_, S_, V, VB, True)
    assert st[0] == 5 and not addr[0].any()      # GSV_ST_INVALID_SIG
    assert st[1] == 0 and bytes(addr[1]) == oracle.keccak256(oracle.secp_pubkey(key)[1:])[12:]


# ---------------------------------------------------------------- host-path argument validation
def test_keccak_rejects_decreasing_offsets(ctx):
    from gsv import _lib
    L = _lib.load()
    data = np.zeros(64, np.uint8)
    off = np.array([0, 40, 8], np.uint64)  # off[2] < off[1]
    out = np.zeros((2, 32), np.uint8)
    rc = L.gsv_keccak256_batch(ctx.handle, ctypes.c_void_p(data.ctypes.data), ctypes.c_void_p(off.ctypes.data), 2,
                               ctypes.c_void_p(out.ctypes.data))
    assert rc == _lib.E_INVALID_ARG


# ---------------------------------------------------------------- *_dev: prepare + graph capture
def test_dev_call_without_prepare_is_refused(ctx):
    import torch
    from gsv import GsvError, _lib
    dev = torch.device("cuda", ctx.device)
    bodies = torch.zeros(3 * 1000 + 17, dtype=torch.uint8, device=dev)
    off = np.array([0, 1000, 2017, 3017], np.uint64)  # a shape no other test prepares
    roots = torch.empty((3, 32), dtype=torch.uint8, device=dev)
    with pytest.raises(GsvError) as e:
        ctx.chunk_root_batch_dev(bodies, off, roots, prepare=False)
    assert e.value.code == _lib.E_NOT_PREPARED
    ctx.chunk_root_prepare(off)
    ctx.chunk_root_batch_dev(bodies, off, roots, prepare=False)
    torch.cuda.synchronize()
    assert bytes(roots[1].cpu().numpy()) == bytes(ctx.chunk_root_batch([bytes(1017)])[0])


def test_dev_calls_capture_into_a_hip_graph(ctx, oracle):
    """Every *_dev entry point, prepared beforehand, records into one HIP graph (no allocation,
    no synchronization inside the capture) and the replay gives the eager results."""
    import torch
    dev = torch.device("cuda", ctx.device)
    rng = np.random.default_rng(4242)
    # ecrecover + keccak
    n = 512
    msg = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    epub = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    eaddr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    ctx.synth_sign_dev(77, msg, sig, epub, eaddr)
    pub = torch.zeros((n, 65), dtype=torch.uint8, device=dev)
    addr = torch.zeros((n, 20), dtype=torch.uint8, device=dev)
    st = torch.full((n,), 9, dtype=torch.uint8, device=dev)
    koff = torch.arange(0, (n + 1) * 32, 32, dtype=torch.int64, device=dev)
    kout = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
    # chunk roots (two lengths + an empty body), POC
    lens = [70000, 70000, 0, 4097]
    h_off = np.zeros(len(lens) + 1, np.uint64)
    h_off[1:] = np.cumsum(lens)
    body_np = rng.integers(0, 256, int(h_off[-1]), dtype=np.uint8)
    bodies = torch.from_numpy(body_np).to(dev)
    roots = torch.zeros((len(lens), 32), dtype=torch.uint8, device=dev)
    salt = bytes(range(1, 21))
    pocs = torch.zeros((len(lens), 32), dtype=torch.uint8, device=dev)
    # pairing (synthetic 4-pair checks + a ragged one)
    nchk = 64
    pin = torch.empty((nchk, 768), dtype=torch.uint8, device=dev)
    pexp = torch.empty((nchk,), dtype=torch.uint8, device=dev)
    ctx.bn256_synth_checks_dev(9, pin, pexp)
    p_off = np.arange(nchk + 1, dtype=np.uint64) * 768
    p_off[-1] -= 5  # last check ragged -> BAD_INPUT
    pver = torch.zeros((nchk,), dtype=torch.uint8, device=dev)
    # DeriveSha over 3 lists
    items = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in rng.integers(1, 150, 90)]
    voff = np.zeros(91, np.uint64)
    voff[1:] = np.cumsum([len(x) for x in items])
    list_off = np.array([0, 40, 40, 90], np.uint64)
    vals = torch.from_numpy(np.frombuffer(b"".join(items) + bytes(8), np.uint8).copy()).to(dev)
    troots = torch.zeros((3, 32), dtype=torch.uint8, device=dev)
    # headers
    nh = 256
    hsid = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hroot = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hper = torch.randint(0, 256, (nh, 32), dtype=torch.uint8, device=dev)
    hprop = torch.randint(0, 256, (nh, 20), dtype=torch.uint8, device=dev)
    hst = torch.zeros((nh,), dtype=torch.uint8, device=dev)
    hhash = torch.zeros((nh, 32), dtype=torch.uint8, device=dev)

    ctx.chunk_root_prepare(h_off)
    ctx.collation_poc_prepare(h_off, salt)
    ctx.pairing_prepare(p_off)
    ctx.derive_sha_prepare(voff, list_off)
    from gsv import _lib
    from gsv._lib import check
    check(_lib.load().gsv_collation_header_prepare(ctx.handle, nh))
    torch.cuda.synchronize()

    def enqueue(s):
        ctx.ecrecover_batch_dev(msg, sig, pub, addr, st, stream=s)
        ctx.keccak256_batch_dev(pub.view(-1)[1:], koff, kout, stream=s)
        ctx.chunk_root_batch_dev(bodies, h_off, roots, stream=s, prepare=False)
        ctx.collation_poc_batch_dev(bodies, h_off, salt, pocs, stream=s, prepare=False)
        ctx.pairing_check_batch_dev(pin, p_off, pver, stream=s, prepare=False)
        ctx.derive_sha_batch_dev(vals, voff, list_off, troots, stream=s, prepare=False)
        ctx.collation_header_verify_batch_dev(hsid, hroot, hper, hprop, sig[:nh], hst, None, hhash, None, stream=s,
                                              prepare=False)

    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    shapes_before = ctx.prepared_shapes()
    with torch.cuda.graph(g, stream=cs):
        enqueue(cs)
    assert ctx.prepared_shapes() == shapes_before  # nothing was built or allocated inside the capture
    g.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in (pub, addr, st, kout, roots, pocs, pver, troots, hst, hhash)]
    for t in (pub, addr, kout, roots, pocs, pver, troots, hst, hhash):
        t.zero_()
    st.fill_(9)
    es = torch.cuda.Stream()
    es.wait_stream(torch.cuda.current_stream())  # the zero / fill above run on the default stream
    enqueue(es)
    es.synchronize()
    eager = (pub, addr, st, kout, roots, pocs, pver, troots, hst, hhash)
    for a, b in zip(got, eager):
        assert torch.equal(a, b)
    # and the results are right
    assert int(st.max()) == 0 and torch.equal(pub, epub) and torch.equal(addr, eaddr)
    bodies_b = [body_np[int(h_off[i]):int(h_off[i + 1])].tobytes() for i in range(len(lens))]
    for i, b in enumerate(bodies_b):
        assert bytes(roots[i].cpu().numpy()) == oracle.derive_sha_bytes(b)
    assert bytes(pocs[3].cpu().numpy()) == oracle.calculate_poc(bodies_b[3], salt)
    want_v = pexp.clone()
    want_v[-1] = _lib.PAIRING_BAD_INPUT
    assert torch.equal(pver, want_v)
    assert bytes(troots[0].cpu().numpy()) == oracle.derive_sha(items[:40])
    assert bytes(troots[1].cpu().numpy()) == oracle.derive_sha([])
    assert bytes(troots[2].cpu().numpy()) == oracle.derive_sha(items[40:90])


def test_pipeline_depth_instances_run_concurrently_and_agree(ctx, oracle):
    """gsv_ctx_set_pipeline_depth: a shape prepared at depth 2 holds two instances, consecutive calls on
    two streams use one each (no ordering between them), and every call's results are the
    single-stream ones; a stream keeps its instance, and depth 1 again leaves later shapes single."""
    import torch
    from gsv import GsvError, _lib
    dev = torch.device("cuda", ctx.device)
    rng = np.random.default_rng(515)
    lens = [65536, 65536, 300, 0, 70000, 65536]  # a shape no other test prepares
    h_off = np.zeros(len(lens) + 1, np.uint64)
    h_off[1:] = np.cumsum(lens)
    body_np = rng.integers(0, 256, int(h_off[-1]), dtype=np.uint8)
    bodies = torch.from_numpy(body_np).to(dev)
    want = ctx.chunk_root_batch([body_np[int(h_off[i]):int(h_off[i + 1])].tobytes() for i in range(len(lens))])
    for i in (2, 3):  # spot-check against the oracle (full-size bodies are covered elsewhere)
        assert bytes(want[i]) == oracle.derive_sha_bytes(body_np[int(h_off[i]):int(h_off[i + 1])].tobytes())
    nchk = 96
    pin = torch.empty((nchk, 768), dtype=torch.uint8, device=dev)
    pexp = torch.empty((nchk,), dtype=torch.uint8, device=dev)
    ctx.bn256_synth_checks_dev(61, pin, pexp)
    p_off = np.arange(nchk + 1, dtype=np.uint64) * 768
    p_off[-1] -= 7  # ragged last check -> BAD_INPUT
    n0, b0 = ctx.prepared_shapes()
    ctx.set_pipeline_depth(2)
    ctx.chunk_root_prepare(h_off)
    ctx.pairing_prepare(p_off)
    ctx.set_pipeline_depth(1)
    torch.cuda.synchronize()  # the synthetic checks were written on the context's stream
    n1, b1 = ctx.prepared_shapes()
    assert n1 == n0 + 2 and b1 > b0
    with pytest.raises(GsvError) as e:
        ctx.set_pipeline_depth(0)
    assert e.value.code == _lib.E_INVALID_ARG
    ss = [torch.cuda.Stream(device=dev) for _ in range(2)]
    roots = [torch.zeros((len(lens), 32), dtype=torch.uint8, device=dev) for _ in range(4)]
    pv = [torch.full((nchk,), 7, dtype=torch.uint8, device=dev) for _ in range(4)]
    for s in ss:
        s.wait_stream(torch.cuda.current_stream())  # the zero / fill above run on the default stream
    for i in range(4):  # calls 0, 2 on stream 0 and 1, 3 on stream 1: the two instances in flight together
        ctx.chunk_root_batch_dev(bodies, h_off, roots[i], stream=ss[i % 2], prepare=False)
        ctx.pairing_check_batch_dev(pin, p_off, pv[i], stream=ss[i % 2], prepare=False)
    for s in ss:
        s.synchronize()
    for i in range(4):
        assert np.array_equal(roots[i].cpu().numpy(), want)
        assert torch.equal(pv[i][:-1], pexp[:-1]) and int(pv[i][-1]) == _lib.PAIRING_BAD_INPUT
    # re-preparing at depth 1 keeps the two-instance shapes (a higher depth is never dropped)
    ctx.chunk_root_prepare(h_off)
    assert ctx.prepared_shapes() == (n1, b1)


@pytest.mark.parametrize("depth", [1, 2])
def test_notary_dev_with_side_stream_captures_into_a_hip_graph(ctx, depth):
    """The notary's _dev call forks its chunk roots onto a side stream (r05: the context's side streams
    sit on hardware queues of their own, CU-masked streams) and joins them by events: the call still
    records into a HIP graph without building anything, and the replay equals the eager results."""
    import torch
    nsh, txs = 3, 256
    dev = torch.device("cuda", ctx.device)
    bodies = torch.empty(nsh * txs * 128, dtype=torch.uint8, device=dev)
    ctx.notary_synth_dev(91, 0, nsh, txs, bodies)
    torch.cuda.synchronize()
    off = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    ctx.set_pipeline_depth(depth)
    try:
        ctx.notary_prepare(off, max_txs=txs)
    finally:
        ctx.set_pipeline_depth(1)
    outs = [torch.zeros((nsh, 32), dtype=torch.uint8, device=dev), torch.zeros((nsh,), dtype=torch.int32, device=dev),
            torch.zeros((nsh, txs // 8), dtype=torch.uint8, device=dev), torch.zeros((nsh, txs), dtype=torch.uint8, device=dev)]
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    shapes_before = ctx.prepared_shapes()
    with torch.cuda.graph(g, stream=cs):
        ctx.notary_validate_shards_dev(bodies, off, outs[0], outs[1], outs[2], None, outs[3], max_txs=txs, stream=cs,
                                       prepare=False)
    assert ctx.prepared_shapes() == shapes_before
    g.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in outs]
    for t in outs:
        t.zero_()
    es = torch.cuda.Stream()
    es.wait_stream(torch.cuda.current_stream())
    ctx.notary_validate_shards_dev(bodies, off, outs[0], outs[1], outs[2], None, outs[3], max_txs=txs, stream=es,
                                   prepare=False)
    es.synchronize()
    for a, b in zip(got, outs):
        assert torch.equal(a, b)
    assert (outs[1].cpu().numpy() == txs).all()
