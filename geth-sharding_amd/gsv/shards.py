"""Shard-ID partition of the notary workload over the GPUs of one node, and the one collective
the path has: an all-gather of fixed-size per-shard validation records.

The reference runs one shard per node (`--shardid`, sharding/node/backend.go:245-284) out of the
SMC's 100 (sharding/contracts/sharding_manager.sol:56).  Here rank r of G owns the contiguous
shard block [floor(100 r / G), floor(100 (r+1) / G)); every rank validates its block locally
(no data-path exchange) and the records {chunk root, tx count, validity bitmap} are all-gathered
so every rank holds the verdict for all shards.  With the "nccl" backend (RCCL over xGMI on ROCm)
the gather runs on the GPU; the same code runs over "gloo" on CPU tensors in the tests.
"""
from __future__ import annotations

ROOT_OFF, NTX_OFF, BM_OFF = 0, 32, 36


def record_bytes(max_txs: int) -> int:
    """root 32 | ntx 4 | bitmap ceil(max_txs/8), padded to 8 bytes"""
    n = BM_OFF + (max_txs + 7) // 8
    return (n + 7) // 8 * 8


def shard_range(rank: int, world: int, n_shards: int):
    return n_shards * rank // world, n_shards * (rank + 1) // world


def shards_per_rank(world: int, n_shards: int) -> int:
    return -(-n_shards // world)


def pack_records(rec, roots, ntx, bitmap):
    """rec: (per_rank, record_bytes) uint8 tensor; roots (n,32) uint8; ntx (n,) int32;
    bitmap (n, bm) uint8 — all on one device.  Rows past n are left as they are."""
    import torch
    n = roots.shape[0]
    rec[:n, ROOT_OFF:ROOT_OFF + 32] = roots
    rec[:n, NTX_OFF:NTX_OFF + 4] = ntx.to(torch.int32).contiguous().view(torch.uint8).view(n, 4)
    rec[:n, BM_OFF:BM_OFF + bitmap.shape[1]] = bitmap
    return rec


def gather_records(rec, world: int, out=None):
    """All-gather every rank's (per_rank, R) record block -> (world * per_rank, R)."""
    import torch
    if world == 1:
        if out is None:
            return rec.clone()
        out.copy_(rec)
        return out
    import torch.distributed as dist
    if out is None:
        out = torch.empty((world * rec.shape[0], rec.shape[1]), dtype=rec.dtype, device=rec.device)
    if dist.get_backend() == "gloo":  # gloo has no all_gather_into_tensor
        parts = [torch.empty_like(rec) for _ in range(world)]
        dist.all_gather(parts, rec)
        out.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(out, rec)
    return out


def unpack_records(gathered, world: int, n_shards: int, max_txs: int):
    """-> (roots (n,32), ntx (n,), bitmap (n, bm)) in shard order"""
    import torch
    per = shards_per_rank(world, n_shards)
    g = gathered.view(world, per, -1)
    rows = torch.cat([g[r, :shard_range(r, world, n_shards)[1] - shard_range(r, world, n_shards)[0]]
                      for r in range(world)])
    bm = (max_txs + 7) // 8
    roots = rows[:, ROOT_OFF:ROOT_OFF + 32]
    ntx = rows[:, NTX_OFF:NTX_OFF + 4].contiguous().view(torch.int32).view(-1)
    bitmap = rows[:, BM_OFF:BM_OFF + bm]
    return roots, ntx, bitmap
