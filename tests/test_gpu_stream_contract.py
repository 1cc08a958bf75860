"""GPU: the NULL-stream contract of the `_dev` entry points (include/gsv.h: stream = NULL runs on the
context's stream, a BLOCKING stream, so it is ordered with the legacy default stream both ways).

The round-4 pairing sweep read verdicts that differed from the generator's truth because a `_dev`
generator ran on a non-blocking context stream while the checker's torch work on the default stream
was not ordered after it (gpurun_out/g3_*.txt; fixed in eb62871, DESIGN §1 "NULL stream").  These
tests pin the contract with no explicit synchronisation between the two sides:

* torch writes the inputs on the default stream behind ~ms of other default-stream work, then the
  library call with stream=None must read the new inputs;
* the library call with stream=None writes its outputs, then torch reads them on the default stream
  at once and must see the new outputs.

Each side is checked for ecrecover (the headline kernel), the chunk root and the pairing check; the
shapes are prepared (and their staging synchronised) beforehand, so only kernel ordering is tested."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def busy():
    """default-stream work that takes a few ms: fills of a 2 GiB buffer"""
    import torch
    buf = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")

    def run():
        for k in range(4):
            buf.fill_(k)
    yield run
    del buf


def _null_stream():
    import torch
    assert torch.cuda.current_stream().cuda_stream == 0, "the test assumes torch's current stream is the null stream"


def _ecrecover_case(ctx, torch, n=1 << 16):
    msg = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    sig = torch.empty((n, 65), dtype=torch.uint8, device="cuda")
    pub = torch.empty((n, 65), dtype=torch.uint8, device="cuda")
    addr = torch.empty((n, 20), dtype=torch.uint8, device="cuda")
    ctx.synth_sign_dev(4242, msg, sig, pub, addr)
    torch.cuda.synchronize()
    return msg, sig, pub, addr


def test_ecrecover_null_stream_reads_after_default_stream_writes(ctx, busy):
    import torch
    _null_stream()
    msg, sig, pub, addr = _ecrecover_case(ctx, torch)
    n = msg.shape[0]
    out_p = torch.empty_like(pub)
    out_a = torch.empty_like(addr)
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    msg2, sig2 = torch.zeros_like(msg), torch.zeros_like(sig)
    ctx.ecrecover_batch_dev(msg2, sig2, out_p, out_a, st)  # warm (comb table) on zero inputs
    torch.cuda.synchronize()
    busy()
    msg2.copy_(msg)
    sig2.copy_(sig)
    ctx.ecrecover_batch_dev(msg2, sig2, out_p, out_a, st)  # stream=None: the context stream
    torch.cuda.synchronize()
    assert torch.equal(out_p, pub) and torch.equal(out_a, addr)
    assert int(st.max()) == 0


def test_ecrecover_default_stream_reads_after_null_stream_call(ctx):
    import torch
    _null_stream()
    msg, sig, pub, addr = _ecrecover_case(ctx, torch)
    n = msg.shape[0]
    out_p = torch.full_like(pub, 0xAA)
    out_a = torch.full_like(addr, 0xAA)
    st = torch.full((n,), 0xAA, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    ctx.ecrecover_batch_dev(msg, sig, out_p, out_a, st)
    got_p, got_a, got_s = out_p.clone(), out_a.clone(), st.clone()  # default stream, no sync
    torch.cuda.synchronize()
    assert torch.equal(got_p, pub) and torch.equal(got_a, addr)
    assert int(got_s.max()) == 0


def _bodies(torch, n=64, size=1 << 16):
    g = torch.Generator(device="cuda").manual_seed(7)
    bodies = torch.randint(0, 256, (n * size,), dtype=torch.uint8, device="cuda", generator=g)
    off = np.arange(n + 1, dtype=np.uint64) * size
    return bodies, off


def test_chunk_root_null_stream_both_ways(ctx, busy):
    import torch
    _null_stream()
    bodies, off = _bodies(torch)
    n = off.shape[0] - 1
    want = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    ctx.chunk_root_batch_dev(bodies, off, want)  # prepares the shape and its staging
    torch.cuda.synchronize()
    ref = ctx.chunk_root_batch([bytes(bodies[int(off[i]):int(off[i + 1])].cpu().numpy()) for i in range(4)])
    assert (want[:4].cpu().numpy() == ref).all()
    # torch -> library
    b2 = torch.zeros_like(bodies)
    roots = torch.full((n, 32), 0xAA, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    busy()
    b2.copy_(bodies)
    ctx.chunk_root_batch_dev(b2, off, roots, prepare=False)
    torch.cuda.synchronize()
    assert torch.equal(roots, want)
    # library -> torch
    roots.fill_(0xAA)
    torch.cuda.synchronize()
    ctx.chunk_root_batch_dev(bodies, off, roots, prepare=False)
    got = roots.clone()
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_pairing_null_stream_both_ways(ctx, busy):
    import torch
    _null_stream()
    n = 4096
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    exp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(5000, pin, exp)
    torch.cuda.synchronize()
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.pairing_prepare(off)
    ver = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    p2 = torch.zeros_like(pin)
    torch.cuda.synchronize()
    # torch -> library: all-zero inputs would read as all-infinity pairs (verdict true everywhere)
    busy()
    p2.copy_(pin)
    ctx.pairing_check_batch_dev(p2, off, ver, prepare=False)
    torch.cuda.synchronize()
    assert torch.equal(ver, exp)
    assert set(exp.cpu().numpy().tolist()) == {0, 1, 2}
    # library -> torch
    ver.fill_(9)
    torch.cuda.synchronize()
    ctx.pairing_check_batch_dev(pin, off, ver, prepare=False)
    got = ver.clone()
    torch.cuda.synchronize()
    assert torch.equal(got, exp)


def test_generator_then_default_stream_check(ctx):
    """the round-4 sweep's own pattern: the configs[4] generator with stream=None, then torch compares
    its output on the default stream with no synchronisation in between"""
    import torch
    _null_stream()
    n = 8192
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    exp = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
    ref_in = torch.empty_like(pin)
    ref_exp = torch.empty_like(exp)
    ctx.bn256_synth_checks_dev(5000, ref_in, ref_exp)
    torch.cuda.synchronize()
    pin.zero_()
    torch.cuda.synchronize()
    ctx.bn256_synth_checks_dev(5000, pin, exp)
    same_in = torch.equal(pin, ref_in)  # default stream, no sync
    same_exp = torch.equal(exp, ref_exp)
    assert same_in and same_exp


def test_pipeline_streams_on_queues_of_their_own(ctx):
    """gsv_stream_create: a pipeline of batches over dedicated-queue streams gives the generator's
    verdicts on every instance, orders after default-stream work (the streams are blocking), and the
    streams are destroyed cleanly; ordering and results only (the timing A/B is
    profiles/r05/ab/stream_sets_*)"""
    import torch
    _null_stream()
    n, depth = 2048, 3
    pin = torch.empty((n, 768), dtype=torch.uint8, device="cuda")
    exp = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ctx.bn256_synth_checks_dev(5001, pin, exp)
    torch.cuda.synchronize()
    off = np.arange(n + 1, dtype=np.uint64) * 768
    ctx.set_pipeline_depth(depth)
    try:
        ctx.pairing_prepare(off)
    finally:
        ctx.set_pipeline_depth(1)
    ss = ctx.pipeline_streams(depth)
    assert len({int(s.cuda_stream) for s in ss}) == depth and all(int(s.cuda_stream) for s in ss)
    vs = [torch.full((n,), 9, dtype=torch.uint8, device="cuda") for _ in range(depth)]
    p2 = torch.zeros_like(pin)
    torch.cuda.synchronize()
    p2.copy_(pin)  # default stream, no explicit synchronisation before the pipelined calls
    for i in range(2 * depth):
        ctx.pairing_check_batch_dev(p2, off, vs[i % depth], stream=ss[i % depth], prepare=False)
    for s in ss:
        s.synchronize()
    ctx.destroy_streams(ss)
    assert all(torch.equal(v, exp) for v in vs)
