"""CPU, world_size 2 over gloo: the row-shard exchange (cyclic ownership, id routing, row replies,
gradient push with DDP averaging) against a single-process computation on the full table."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, V, D, q):
    sys.path.insert(0, ROOT)
    import __graft_entry__
    asme = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = asme.sharded.RowShardExchange(V)
        g = torch.Generator().manual_seed(0)
        table = torch.randn(V, D, generator=g)                       # the logical full table (same on all)
        shard = table[rank::world].clone()                            # cyclic row shard
        assert shard.shape[0] == asme.sharded.shard_rows(V, world, rank)
        gr = torch.Generator().manual_seed(100 + rank)
        unique = torch.randperm(V, generator=gr)[: 17 + 5 * rank]     # this rank's distinct ids
        st = ex.request(unique)
        assert int((st.recv_local >= shard.shape[0]).sum()) == 0
        rows = ex.reply_rows(st, shard[st.recv_local])                # send order: row j <-> unique[order[j]]
        ok_rows = torch.equal(rows, table[unique[st.order]]) and torch.equal(rows[st.pos], table[unique])
        ok_rows = ok_rows and bool((unique[st.order] % world == torch.sort(unique[st.order] % world).values).all())
        # gradient push: owners receive every requester's rows, averaged over ranks
        grad = torch.randn(len(unique), D, generator=gr)
        recv = ex.push_grads(st, grad[st.order])
        acc = torch.zeros_like(shard)
        acc.index_add_(0, st.recv_local, recv / world)
        # reference: every rank's (unique, grad) scattered into the full table, then sliced
        all_u = [torch.empty(0, dtype=torch.int64)] * world
        all_g = [None] * world
        objs = [None] * world
        dist.all_gather_object(objs, (unique, grad))
        full = torch.zeros(V, D)
        for u, gg in objs:
            full.index_add_(0, u, gg / world)
        ok_grad = torch.allclose(acc, full[rank::world], atol=1e-6)
        q.put((rank, ok_rows, ok_grad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_shard_exchange_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 101, 8, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok_r and ok_g for _, ok_r, ok_g in res), res
