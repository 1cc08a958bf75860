"""The native shard partition + RCCL all-gather entry point (gsv.h gsv_notary_validate_partition,
SURVEY.md §8e; reference partition sharding/node/backend.go:245-284): on one GPU as a one-rank RCCL
communicator, every shard's gathered record equals gsv_notary_validate_shards' on the same bodies.
(More ranks need more GPUs: the driver's 8-GPU bench runs the partition through torch.distributed;
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
