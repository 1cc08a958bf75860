"""CPU tests of the multi-GPU path's host logic: the shard-ID partition and the all-gather of
per-shard records (gsv.shards), run with world_size 2 and 3 over gloo on 127.0.0.1 — the same
code bench.py runs over RCCL with one process per GPU."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_SHARDS, MAX_TXS = 100, 8192


def test_partition_covers_all_shards():
    from gsv import shards as SH
    for g in range(1, 9):
        ranges = [SH.shard_range(r, g, N_SHARDS) for r in range(g)]
        assert ranges[0][0] == 0 and ranges[-1][1] == N_SHARDS
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(g - 1))
        sizes = [b - a for a, b in ranges]
        assert max(sizes) - min(sizes) <= 1 and max(sizes) <= SH.shards_per_rank(g, N_SHARDS)
    assert SH.record_bytes(MAX_TXS) == 1064


def _fake_records(lo, hi):
    n = hi - lo
    ids = torch.arange(lo, hi, dtype=torch.int64)
    roots = (ids.view(n, 1) * 7 + torch.arange(32).view(1, 32)).to(torch.uint8)
    ntx = (ids * 3 + 1).to(torch.int32)
    bitmap = ((ids.view(n, 1) + torch.arange(MAX_TXS // 8).view(1, -1)) % 251).to(torch.uint8)
    return roots, ntx, bitmap


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        from gsv import shards as SH
        dist.init_process_group("gloo", rank=rank, world_size=world)
        lo, hi = SH.shard_range(rank, world, N_SHARDS)
        per = SH.shards_per_rank(world, N_SHARDS)
        rec = torch.zeros((per, SH.record_bytes(MAX_TXS)), dtype=torch.uint8)
        SH.pack_records(rec, *_fake_records(lo, hi))
        g = SH.gather_records(rec, world)
        roots, ntx, bitmap = SH.unpack_records(g, world, N_SHARDS, MAX_TXS)
        want = _fake_records(0, N_SHARDS)
        ok = torch.equal(roots, want[0]) and torch.equal(ntx, want[1]) and torch.equal(bitmap, want[2])
        q.put((rank, ok))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_gather_records_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r for r, _ in res) == list(range(world))
    assert all(ok is True for _, ok in res), res
