"""GPU: who owns the library's HIP objects, and what happens at process exit.

r05 record: `gpurun_out/r05l/sets_traced.txt` — a pairing sweep that left eight CU-masked streams and the
default context to the runtime's static destructors died with SIGSEGV in `__cxa_finalize` after rocprofv3
finalised.  Since r06 the context owns its dedicated-queue streams (`gsv_stream_create` refuses past
GSV_MAX_STREAMS, `gsv_stream_destroy` refuses foreign handles, `gsv_ctx_destroy` destroys what is left),
each prepared shape owns its side streams, and the Python package closes every live context at
interpreter exit (atexit), before the HIP runtime tears down."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = textwrap.dedent("""
    import ctypes, os, sys
    sys.path.insert(0, os.path.join(sys.argv[1], "geth-sharding_amd"))
    import numpy as np
    import torch
    import gsv
    from gsv import _lib
    ctx = gsv.default_context()
    # a pipeline three deep on dedicated-queue streams, shapes prepared three deep (notary side streams)
    ss = ctx.pipeline_streams(3)
    n = 1024
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    pexp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(77, pin, pexp)
    torch.cuda.synchronize()
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.set_pipeline_depth(3)
    ctx.pairing_prepare(off)
    nsh, txs = 2, 128
    bodies = torch.empty(nsh * txs * 128, dtype=torch.uint8, device="cuda")
    ctx.notary_synth_dev(5, 0, nsh, txs, bodies)
    torch.cuda.synchronize()
    noff = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    ctx.notary_prepare(noff, max_txs=txs)
    ctx.set_pipeline_depth(1)
    pv = [torch.empty((n,), dtype=torch.uint8, device="cuda") for _ in range(3)]
    for i in range(3):
        ctx.pairing_check_batch_dev(pin, off, pv[i], stream=ss[i], prepare=False)
    r = torch.empty((nsh, 32), dtype=torch.uint8, device="cuda")
    c = torch.empty((nsh,), dtype=torch.int32, device="cuda")
    b = torch.empty((nsh, txs // 8), dtype=torch.uint8, device="cuda")
    ctx.notary_validate_shards_dev(bodies, noff, r, c, b, None, None, max_txs=txs, stream=ss[0], prepare=False)
    torch.cuda.synchronize()
    assert all(torch.equal(v, pexp) for v in pv)
    assert (c.cpu().numpy() == txs).all()
    u, s = ctx.stream_count()
    assert u == 3 and s == 3, (u, s)
    # a second context whose caller-side streams are never destroyed: gsv_ctx_destroy must take them
    L = _lib.load()
    h = ctypes.c_void_p()
    assert L.gsv_ctx_create(0, ctypes.byref(h)) == 0
    for _ in range(2):
        q = ctypes.c_void_p()
        assert L.gsv_stream_create(h, ctypes.byref(q)) == 0
    L.gsv_ctx_destroy(h)
    print("child ok", flush=True)
    # no cleanup: the default context, its three pipeline streams and the prepared shapes' side streams
    # are left to interpreter exit
""")


def test_process_exit_with_live_streams_and_default_context():
    """A child process makes pipeline streams, shapes with side streams and the default context, runs a
    pairing batch and a notary step on them, and returns without any cleanup: it must exit with rc 0."""
    p = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, f"rc {p.returncode}\nstdout:\n{p.stdout[-2000:]}\nstderr:\n{p.stderr[-4000:]}"
    assert "child ok" in p.stdout


def test_stream_cap_and_foreign_handles(ctx):
    """gsv_stream_create refuses the (GSV_MAX_STREAMS + 1)-th live stream of a context; gsv_stream_destroy
    refuses a handle the context did not create (and a second destroy of one it did)."""
    import ctypes
    import gsv
    from gsv import _lib
    L = _lib.load()
    c2 = gsv.Context(ctx.device)
    try:
        made = []
        for _ in range(_lib.MAX_STREAMS):
            q = ctypes.c_void_p()
            assert L.gsv_stream_create(c2.handle, ctypes.byref(q)) == 0
            made.append(q.value)
        q = ctypes.c_void_p()
        assert L.gsv_stream_create(c2.handle, ctypes.byref(q)) == _lib.E_INVALID_ARG
        assert q.value is None
        assert c2.stream_count()[0] == _lib.MAX_STREAMS
        # a handle of another context (and a torch stream) is not this context's to destroy
        other = ctx.pipeline_streams(1)
        try:
            assert L.gsv_stream_destroy(c2.handle, int(other[0].cuda_stream)) == _lib.E_INVALID_ARG
        finally:
            ctx.destroy_streams(other)
        import torch
        ts = torch.cuda.Stream()
        assert L.gsv_stream_destroy(c2.handle, int(ts.cuda_stream)) == _lib.E_INVALID_ARG
        assert L.gsv_stream_destroy(c2.handle, made[0]) == 0
        assert L.gsv_stream_destroy(c2.handle, made[0]) == _lib.E_INVALID_ARG
        assert c2.stream_count()[0] == _lib.MAX_STREAMS - 1
        with pytest.raises(gsv.GsvError):
            c2.pipeline_streams(_lib.MAX_STREAMS)  # the Python side checks the cap before creating any
    finally:
        c2.close()  # destroys the seven streams still live


def _notary_case(torch, dev, nsh, txs, seed):
    bodies = torch.empty(nsh * txs * 128, dtype=torch.uint8, device=dev)
    return bodies, np.arange(nsh + 1, dtype=np.uint64) * txs * 128


def _notary_outs(torch, dev, nsh, txs):
    return [torch.zeros((nsh, 32), dtype=torch.uint8, device=dev), torch.zeros((nsh,), dtype=torch.int32, device=dev),
            torch.zeros((nsh, txs // 8), dtype=torch.uint8, device=dev),
            torch.zeros((nsh, txs), dtype=torch.uint8, device=dev)]


def test_side_streams_are_per_shape_and_bounded():
    """Each prepared notary shape owns one side stream per pipeline instance; a retired shape gives its
    side streams back; past 8 live side streams a newly prepared shape takes the least recently used
    shape's (which then runs its chunk roots after its transactions on the caller's stream); every shape
    gives the same results as a fresh context's."""
    import torch
    import gsv
    c = gsv.Context(0)
    try:
        dev = torch.device("cuda", c.device)
        txs = 128
        cases = []
        for nsh in (2, 3, 4):  # three different shapes (body offsets differ)
            bodies, off = _notary_case(torch, dev, nsh, txs, 0)
            c.notary_synth_dev(31 + nsh, 0, nsh, txs, bodies)
            cases.append((nsh, bodies, off))
        torch.cuda.synchronize()
        c.set_pipeline_depth(3)
        c.notary_prepare(cases[0][2], max_txs=txs)
        assert c.stream_count()[1] == 3
        c.set_pipeline_depth(4)  # re-prepare retires the depth-3 shape: its three side streams go
        c.notary_prepare(cases[0][2], max_txs=txs)
        assert c.stream_count()[1] == 4
        c.notary_prepare(cases[1][2], max_txs=txs)
        assert c.stream_count()[1] == 8
        c.notary_prepare(cases[2][2], max_txs=txs)  # past the bound: takes the LRU shape's (case 0's) four
        assert c.stream_count()[1] == 8
        c.set_pipeline_depth(1)
        ref = gsv.default_context()
        for nsh, bodies, off in cases:
            got = _notary_outs(torch, dev, nsh, txs)
            want = _notary_outs(torch, dev, nsh, txs)
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            c.notary_validate_shards_dev(bodies, off, got[0], got[1], got[2], None, got[3], max_txs=txs, stream=st,
                                         prepare=False)
            ref.notary_validate_shards_dev(bodies, off, want[0], want[1], want[2], None, want[3], max_txs=txs,
                                           stream=st)
            st.synchronize()
            for a, b in zip(got, want):
                assert torch.equal(a, b)
            assert (got[1].cpu().numpy() == txs).all()
    finally:
        c.close()


def test_capture_beside_uncaptured_calls_of_other_shapes(ctx):
    """while a notary _dev call is being captured on stream A, uncaptured calls of
    OTHER shapes — a second notary shape (side streams of its own) and a pairing batch — run on stream B
    before EndCapture.  Neither may join or break A's capture; the replay and the eager calls give the
    same results."""
    import torch
    dev = torch.device("cuda", ctx.device)
    txs = 256
    (ba, offa), (bb, offb) = _notary_case(torch, dev, 3, txs, 0), _notary_case(torch, dev, 5, txs, 0)
    ctx.notary_synth_dev(61, 0, 3, txs, ba)
    ctx.notary_synth_dev(62, 0, 5, txs, bb)
    n = 2048
    pin = torch.empty((n, 768), dtype=torch.uint8, device=dev)
    pexp = torch.empty((n,), dtype=torch.uint8, device=dev)
    ctx.bn256_synth_checks_dev(63, pin, pexp)
    torch.cuda.synchronize()
    poff = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.set_pipeline_depth(2)
    try:
        ctx.notary_prepare(offa, max_txs=txs)
        ctx.notary_prepare(offb, max_txs=txs)
        ctx.pairing_prepare(poff)
    finally:
        ctx.set_pipeline_depth(1)
    oa, ob = _notary_outs(torch, dev, 3, txs), _notary_outs(torch, dev, 5, txs)
    pv = torch.zeros((n,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sa, capture_error_mode="thread_local"):
        ctx.notary_validate_shards_dev(ba, offa, oa[0], oa[1], oa[2], None, oa[3], max_txs=txs, stream=sa,
                                       prepare=False)
        # uncaptured work of other shapes on another stream, inside the capture window
        ctx.notary_validate_shards_dev(bb, offb, ob[0], ob[1], ob[2], None, ob[3], max_txs=txs, stream=sb,
                                       prepare=False)
        ctx.pairing_check_batch_dev(pin, poff, pv, stream=sb, prepare=False)
    sb.synchronize()
    assert torch.equal(pv, pexp)
    assert (ob[1].cpu().numpy() == txs).all()
    g.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in oa]
    ea = _notary_outs(torch, dev, 3, txs)
    es = torch.cuda.Stream()
    ctx.notary_validate_shards_dev(ba, offa, ea[0], ea[1], ea[2], None, ea[3], max_txs=txs, stream=es, prepare=False)
    es.synchronize()
    for a, b in zip(got, ea):
        assert torch.equal(a, b)
    assert (got[1].cpu().numpy() == txs).all()


_CHILD_NO_SIDE = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, os.path.join(sys.argv[1], "geth-sharding_amd"))
    import numpy as np
    import torch
    import gsv
    ctx = gsv.default_context()
    nsh, txs = 3, 256
    bodies = torch.empty(nsh * txs * 128, dtype=torch.uint8, device="cuda")
    exp = torch.empty(nsh * txs, dtype=torch.uint8, device="cuda")
    ctx.notary_synth_dev(44, 0, nsh, txs, bodies, exp)
    torch.cuda.synchronize()
    off = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    ctx.set_pipeline_depth(3)
    ctx.notary_prepare(off, max_txs=txs)
    ctx.set_pipeline_depth(1)
    assert ctx.stream_count() == (0, 0), ctx.stream_count()
    ss = ctx.pipeline_streams(3)
    outs = []
    for i in range(6):
        o = [torch.zeros((nsh, 32), dtype=torch.uint8, device="cuda"), torch.zeros((nsh,), dtype=torch.int32, device="cuda"),
             torch.zeros((nsh, txs // 8), dtype=torch.uint8, device="cuda"), torch.zeros((nsh, txs), dtype=torch.uint8, device="cuda")]
        ctx.notary_validate_shards_dev(bodies, off, o[0], o[1], o[2], None, o[3], max_txs=txs, stream=ss[i % 3],
                                       prepare=False)
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o[3].view(-1), exp) and (o[1].cpu().numpy() == txs).all()
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[2], outs[0][2])
    print("roots", outs[0][0].cpu().numpy().tobytes().hex(), flush=True)
""")


def test_no_side_streams_runs_the_chunk_roots_serially(ctx):
    """GSV_MAX_SIDE_STREAMS=0 (the leg-only profile pass, tools/profile_round.sh): a notary shape gets no
    side streams, its steps run the chunk roots after the transactions on the caller's stream, six
    pipelined steps give the construction's statuses, and the roots equal this process's (forked) ones."""
    import torch
    env = dict(os.environ, GSV_MAX_SIDE_STREAMS="0")
    p = subprocess.run([sys.executable, "-c", _CHILD_NO_SIDE, ROOT], capture_output=True, text=True, timeout=240,
                       env=env)
    assert p.returncode == 0, f"rc {p.returncode}\nstdout:\n{p.stdout[-2000:]}\nstderr:\n{p.stderr[-4000:]}"
    roots = [l.split()[1] for l in p.stdout.splitlines() if l.startswith("roots ")][0]
    nsh, txs = 3, 256
    bodies = torch.empty(nsh * txs * 128, dtype=torch.uint8, device="cuda")
    ctx.notary_synth_dev(44, 0, nsh, txs, bodies)
    torch.cuda.synchronize()
    off = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    o = [torch.zeros((nsh, 32), dtype=torch.uint8, device="cuda"), torch.zeros((nsh,), dtype=torch.int32, device="cuda"),
         torch.zeros((nsh, txs // 8), dtype=torch.uint8, device="cuda")]
    ctx.notary_validate_shards_dev(bodies, off, o[0], o[1], o[2], None, None, max_txs=txs)
    torch.cuda.synchronize()
    assert o[0].cpu().numpy().tobytes().hex() == roots
