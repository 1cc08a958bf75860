"""The native shard partition + RCCL all-gather entry point (gsv.h gsv_notary_validate_partition,
SURVEY.md §8e; reference partition sharding/node/backend.go:245-284): on one GPU as a one-rank RCCL
communicator, every shard's gathered record equals gsv_notary_validate_shards' on the same bodies.
(More RCCL ranks need more GPUs: the driver's 8-GPU bench runs the partition through torch.distributed;
the record layout and block arithmetic are shared with gsv/shards.py and tested with gloo.)"""
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


def _rank_worker(rank, world, port, nsh, txs, q):
    """one rank process: validate this rank's shard block on the GPU, pack its records on the GPU,
    all-gather them over gloo (the collective bench.py runs over RCCL), check every shard's record
    against a whole-batch validation in this process"""
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
        g_root, g_ntx, g_bm = SH.unpack_records(g, world, nsh, txs)
        # the whole batch validated in this process
        allb = torch.empty((nsh * txs * 128,), dtype=torch.uint8, device=dev)
        ctx.notary_synth_dev(4242, 0, nsh, txs, allb)
        torch.cuda.synchronize()
        flat = allb.cpu().numpy()
        want = ctx.notary_validate_shards([flat[i * txs * 128:(i + 1) * txs * 128].tobytes() for i in range(nsh)],
                                          max_txs=txs)
        ok = (np.array_equal(g_root.numpy(), want[0]) and np.array_equal(g_ntx.numpy(), want[1])
              and np.array_equal(g_bm.numpy(), want[2]))
        q.put((rank, ok))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_on_one_gpu_validate_blocks_and_gather(world):
    """world rank processes on the one GPU: each validates its shard block
    (sharding/node/backend.go:245-284 partition) and the gathered records equal a whole-batch
    validation: the GPU validation composed with the partition's all-gather, across processes."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    nsh, txs = 7, 256
    ps = [ctxm.Process(target=_rank_worker, args=(r, world, port, nsh, txs, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=100) for _ in range(world))
    for p in ps:
        p.join(timeout=30)
    assert res == {r: True for r in range(world)}, res
