"""The native shard partition + RCCL all-gather entry points (gsv.h gsv_notary_validate_partition[_dev],
gsv_notary_partition_pack_dev / _unpack_dev; reference partition
sharding/node/backend.go:245-284).

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so on the one-GPU box:
  * the RCCL entry points run as a one-rank communicator against gsv_notary_validate_shards, including
    the rank-local failure path (the rank still reaches the collective and reports its status);
  * 2 and 3 rank processes run the same pack -> all-gather -> unpack through the C ABI with the
    all-gather over gloo (host): the block layout and the unpack offsets of ranks q > 0 are the ones the
    RCCL path uses (bench.py --gpus N runs gsv_notary_validate_partition_dev over RCCL)."""
import numpy as np
import pytest

import gsv

pytestmark = pytest.mark.gpu


def test_partition_one_rank_equals_local_validation(ctx):
    import torch
    nsh, txs = 12, 256
    dev = torch.device("cuda", ctx.device)
    bodies_t = torch.empty(nsh * txs * 128, dtype=torch.uint8, device=dev)
    ctx.notary_synth_dev(77, 0, nsh, txs, bodies_t)
    torch.cuda.synchronize()
    flat = bodies_t.cpu().numpy()
    bodies = [flat[i * txs * 128:(i + 1) * txs * 128].tobytes() for i in range(nsh)]
    uid = gsv.comm_unique_id()
    assert len(uid) == 128
    ctx.comm_init(uid, 1, 0)
    assert ctx.comm_info() == (1, 0)
    want = ctx.notary_validate_shards(bodies, max_txs=txs)
    got = ctx.notary_validate_partition(bodies, nsh, max_txs=txs, want_senders=True, want_status=True)
    for a, b in zip(want, got):
        assert np.array_equal(a, b)
    assert (got[1] == txs).all() and got[2].any()
    # a rank with an empty block still receives every shard's record (here: 0 shards of 0)
    r = ctx.notary_validate_partition([], 0, max_txs=txs)
    assert r[0].shape == (0, 32)
    # device-resident form on the same communicator
    off = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    root = torch.zeros((nsh, 32), dtype=torch.uint8, device=dev)
    ntx = torch.zeros((nsh,), dtype=torch.int32, device=dev)
    bm = torch.zeros((nsh, txs // 8), dtype=torch.uint8, device=dev)
    rst = torch.full((1,), -99, dtype=torch.int32, device=dev)
    ctx.notary_validate_partition_dev(bodies_t, off, nsh, root, ntx, bm, rank_status_t=rst, max_txs=txs)
    torch.cuda.synchronize()
    assert np.array_equal(root.cpu().numpy(), want[0]) and np.array_equal(bm.cpu().numpy(), want[2])
    assert (ntx.cpu().numpy() == txs).all() and int(rst[0]) == 0


@pytest.mark.parametrize("streams", ["torch", "dedicated"])
def test_partition_dev_pipelined_on_two_streams(ctx, streams):
    """Consecutive partition calls kept in flight on two streams (pipeline depth 2): each call's records
    equal the whole-batch validation.  At N > 1 the library orders their all-gathers on the
    communicator (a one-rank RCCL communicator here).  `dedicated`: the streams bench.py's notary leg
    uses (gsv_stream_create, a hardware queue each), so the RCCL all-gather runs on them here before
    the driver's multi-GPU run does."""
    import torch
    nsh, txs = 13, 512
    dev = torch.device("cuda", ctx.device)
    bodies_t = torch.empty(nsh * txs * 128, dtype=torch.uint8, device=dev)
    ctx.notary_synth_dev(78, 0, nsh, txs, bodies_t)
    torch.cuda.synchronize()
    flat = bodies_t.cpu().numpy()
    want = ctx.notary_validate_shards([flat[i * txs * 128:(i + 1) * txs * 128].tobytes() for i in range(nsh)],
                                      max_txs=txs)
    ctx.comm_init(gsv.comm_unique_id(), 1, 0)
    off = np.arange(nsh + 1, dtype=np.uint64) * txs * 128
    ctx.set_pipeline_depth(2)
    try:
        ctx.notary_partition_prepare(off, nsh, 1, 0, max_txs=txs)
    finally:
        ctx.set_pipeline_depth(1)
    ss = ctx.pipeline_streams(2) if streams == "dedicated" else [torch.cuda.Stream(device=dev) for _ in range(2)]
    outs = [(torch.zeros((nsh, 32), dtype=torch.uint8, device=dev), torch.zeros((nsh,), dtype=torch.int32, device=dev),
             torch.zeros((nsh, txs // 8), dtype=torch.uint8, device=dev),
             torch.full((1,), -99, dtype=torch.int32, device=dev)) for _ in range(6)]
    for s_ in ss:
        s_.wait_stream(torch.cuda.current_stream())
    for i, (root, ntx, bm, rst) in enumerate(outs):
        ctx.notary_validate_partition_dev(bodies_t, off, nsh, root, ntx, bm, rank_status_t=rst, max_txs=txs,
                                          stream=ss[i % 2], prepare=False)
    torch.cuda.synchronize()
    ctx.destroy_streams(ss)
    for root, ntx, bm, rst in outs:
        assert np.array_equal(root.cpu().numpy(), want[0]) and np.array_equal(bm.cpu().numpy(), want[2])
        assert (ntx.cpu().numpy() == txs).all() and int(rst[0]) == 0


def test_partition_local_failure_still_joins_the_collective(ctx):
    """a rank-local failure returns its status after the all-gather, not before it."""
    import torch
    from gsv._lib import GsvError, E_TOO_LARGE, E_NOT_PREPARED
    txs = 256
    dev = torch.device("cuda", ctx.device)
    ctx.comm_init(gsv.comm_unique_id(), 1, 0)
    # host form: a body over 2^20 bytes (sharding/collation.go:45)
    with pytest.raises(GsvError) as e:
        ctx.notary_validate_partition([bytes((1 << 20) + 1)], 1, max_txs=txs)
    assert e.value.code == E_TOO_LARGE
    # device form, never prepared for these offsets: the rank status says why
    off = np.array([0, txs * 128], np.uint64)
    nb = torch.zeros(txs * 128, dtype=torch.uint8, device=dev)
    root = torch.full((1, 32), 7, dtype=torch.uint8, device=dev)
    ntx = torch.zeros((1,), dtype=torch.int32, device=dev)
    bm = torch.zeros((1, txs // 8), dtype=torch.uint8, device=dev)
    rst = torch.zeros((1,), dtype=torch.int32, device=dev)
    with pytest.raises(GsvError) as e:
        ctx.notary_validate_partition_dev(nb, off + 16, 1, root, ntx, bm, rank_status_t=rst, max_txs=txs,
                                          prepare=False)
    assert e.value.code == E_NOT_PREPARED
    torch.cuda.synchronize()
    assert int(rst[0]) == E_NOT_PREPARED and int(root.sum()) == 0 and int(ntx[0]) == 0
    # and the context still works afterwards
    ctx.notary_validate_partition_dev(nb, off, 1, root, ntx, bm, rank_status_t=rst, max_txs=txs)
    torch.cuda.synchronize()
    assert int(rst[0]) == 0 and int(ntx[0]) == 0  # an all-zero body holds no blobs


def _rank_worker(rank, world, port, nsh, txs, q):
    """one rank process: validate this rank's shard block and pack its record block through the C ABI
    (gsv_notary_partition_pack_dev), all-gather the blocks over gloo (the step RCCL does in
    gsv_notary_validate_partition_dev), unpack them through the C ABI (gsv_notary_partition_unpack_dev),
    and check every shard's record against a whole-batch validation in this process; the torch form
    of the same records (gsv/shards.py) must agree."""
    import os
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        import gsv as G
        from gsv import shards as SH
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ctx = G.default_context()
        dev = torch.device("cuda", ctx.device)
        lo, hi = SH.shard_range(rank, world, nsh)
        n = hi - lo
        nb = torch.empty((max(n, 1) * txs * 128,), dtype=torch.uint8, device=dev)
        if n:
            ctx.notary_synth_dev(4242, lo, n, txs, nb)
        off = np.arange(n + 1, dtype=np.uint64) * txs * 128
        root = torch.zeros((n, 32), dtype=torch.uint8, device=dev)
        cnt = torch.zeros((n,), dtype=torch.int32, device=dev)
        bm = torch.zeros((n, txs // 8), dtype=torch.uint8, device=dev)
        if n:
            ctx.notary_validate_shards_dev(nb, off, root, cnt, bm, None, None, max_txs=txs)
        torch.cuda.synchronize()
        per = SH.shards_per_rank(world, nsh)
        rec = torch.zeros((per, SH.record_bytes(txs)), dtype=torch.uint8, device=dev)
        SH.pack_records(rec, root, cnt, bm)
        g = SH.gather_records(rec.cpu(), world)  # gloo: host tensors
        t_root, t_ntx, t_bm = SH.unpack_records(g, world, nsh, txs)
        # the C-ABI form: pack -> all-gather (gloo here, RCCL in the combined entry point) -> unpack
        B = G.partition_block_bytes(nsh, world, txs)
        blk = torch.zeros((B,), dtype=torch.uint8, device=dev)
        ctx.notary_partition_pack_dev(nb, off, nsh, world, rank, blk, max_txs=txs)
        torch.cuda.synchronize()
        parts = [torch.empty((B,), dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, blk.cpu())
        allb_t = torch.cat(parts).to(dev)
        torch.cuda.synchronize()  # the unpack runs on the context's stream
        g_root = torch.zeros((nsh, 32), dtype=torch.uint8, device=dev)
        g_ntx = torch.zeros((nsh,), dtype=torch.int32, device=dev)
        g_bm = torch.zeros((nsh, txs // 8), dtype=torch.uint8, device=dev)
        g_rst = torch.full((world,), -1, dtype=torch.int32, device=dev)
        ctx.notary_partition_unpack_dev(allb_t, nsh, world, g_root, g_ntx, g_bm, g_rst, max_txs=txs)
        torch.cuda.synchronize()
        g_root, g_ntx, g_bm = g_root.cpu(), g_ntx.cpu(), g_bm.cpu()
        assert (g_rst.cpu() == 0).all(), f"rank statuses {g_rst.cpu().tolist()}"
        for nm, a, b in (("root", g_root, t_root), ("ntx", g_ntx, t_ntx), ("bitmap", g_bm, t_bm)):
            bad = [i for i in range(nsh) if not torch.equal(a[i], b[i])]
            assert not bad, f"C-ABI vs torch gather: {nm} differs at shards {bad[:8]} (this rank: {lo}..{hi - 1})"
        # the whole batch validated in this process
        allb = torch.empty((nsh * txs * 128,), dtype=torch.uint8, device=dev)
        ctx.notary_synth_dev(4242, 0, nsh, txs, allb)
        torch.cuda.synchronize()
        flat = allb.cpu().numpy()
        want = ctx.notary_validate_shards([flat[i * txs * 128:(i + 1) * txs * 128].tobytes() for i in range(nsh)],
                                          max_txs=txs)
        ok = True
        for nm, a, b in (("root", g_root.numpy(), want[0]), ("ntx", g_ntx.numpy(), want[1]), ("bitmap", g_bm.numpy(), want[2])):
            bad = [i for i in range(nsh) if not np.array_equal(a[i], b[i])]
            if bad:
                ok = f"gathered vs whole batch: {nm} differs at shards {bad[:8]} (this rank: {lo}..{hi - 1})"
                break
        q.put((rank, ok))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world,nsh,txs", [(2, 7, 256), (3, 7, 256), (4, 100, 64), (8, 100, 64)])
def test_ranks_on_one_gpu_validate_blocks_and_gather(world, nsh, txs):
    """world rank processes on the one GPU: each validates its shard block
    (sharding/node/backend.go:245-284 partition) and the gathered records equal a whole-batch
    validation: the GPU validation composed with the partition's all-gather, across processes.
    (4, 100) and (8, 100) are configs[3]'s geometry at N = 4 and 8: 25 shards per rank, and 12 or 13
    shards per rank in blocks padded to 13 records, unpacked at the offsets of ranks 1..7."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    ps = [ctxm.Process(target=_rank_worker, args=(r, world, port, nsh, txs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    assert res == {r: True for r in range(world)}, res
