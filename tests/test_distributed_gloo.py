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


def _worker(rank, world, port, V, D, split, q):
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
        # split: two classes (overlap_negatives), the first 5 + rank unique ids and the rest, each routed by owner
        sp = torch.tensor([5 + rank], dtype=torch.int32) if split else None
        st = ex.request(unique, split=sp)
        assert int((st.recv_local >= shard.shape[0]).sum()) == 0
        rows = ex.reply_rows(st, shard[st.recv_local], async_second=split)  # send order: row j <-> unique[order[j]]
        assert st.work is None  # (CPU gloo: complete on return)
        ok_rows = torch.equal(rows, table[unique[st.order]]) and torch.equal(rows[st.pos], table[unique])
        key = unique[st.order] % world
        if split:  # class-major: the first class's ids (slots < split) by owner, then the rest by owner
            cls = (st.order >= 5 + rank).to(torch.int64)
            key = key + world * cls
            ok_rows = ok_rows and int(st.classes[0][0] + sum(st.classes[0][1:])) == 5 + rank
        ok_rows = ok_rows and bool((key == torch.sort(key).values).all())
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


@pytest.mark.parametrize("world,split", [(2, False), (3, False), (2, True), (3, True)])
def test_row_shard_exchange_gloo(world, split):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 101, 8, split, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok_r and ok_g for _, ok_r, ok_g in res), res


# ---------------------------------------------------------------------------------------- data parallel
class _Toy(torch.nn.Module):
    """stand-in for a recommender module (no HIP kernels on CPU): three layers, one of them unused on some steps"""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(6, 64)
        self.b = torch.nn.Linear(64, 64)
        self.unused = torch.nn.Linear(3, 3)

    def loss(self, x, use_unused):
        y = self.b(torch.tanh(self.a(x))).pow(2).mean()
        if use_unused:
            y = y + self.unused(x[:, :3]).sum()
        return y


def _dp_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import __graft_entry__
    asme = __graft_entry__.load_package()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = _Toy()
        # tiny buckets: several collectives per step, launched from the backward hooks in a fixed order
        red = asme.dataparallel.GradientAllReduce(m, bucket_bytes=4096)
        g = torch.Generator().manual_seed(7)
        xs = [torch.randn(5, 6, generator=g) for _ in range(world)]  # every rank's slice (identical on all ranks)
        use_unused = rank == 0                                         # a parameter with a gradient on one rank only
        m.loss(xs[rank], use_unused).backward()
        red.finish()
        got = {n: p.grad.clone() for n, p in m.named_parameters()}
        # DDP semantics: the mean of the per-rank gradients of the per-rank losses
        want = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
        for r in range(world):
            ref = _Toy()
            ref.loss(xs[r], r == 0).backward()
            for n, p in ref.named_parameters():
                if p.grad is not None:
                    want[n] += p.grad / world
        err = max(float((got[n] - want[n]).abs().max()) for n in got)
        # gradient accumulation (accumulate_grad_batches = 2): the first micro-batch inside no_sync(), the
        # second outside; the average over ranks of each rank's accumulated gradient
        m.zero_grad(set_to_none=True)
        x2 = [torch.randn(5, 6, generator=g) for _ in range(world)]
        with red.no_sync():
            m.loss(xs[rank], use_unused).backward()
        m.loss(x2[rank], use_unused).backward()
        red.finish()
        want2 = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
        for r in range(world):
            ref = _Toy()
            ref.loss(xs[r], r == 0).backward()
            ref.loss(x2[r], r == 0).backward()
            for n, p in ref.named_parameters():
                if p.grad is not None:
                    want2[n] += p.grad / world
        err = max(err, max(float((p.grad - want2[n]).abs().max()) for n, p in m.named_parameters()))
        # a second backward without no_sync() must raise instead of silently averaging only the first
        m.zero_grad(set_to_none=True)
        m.loss(xs[rank], True).backward()
        try:
            m.loss(xs[rank], True).backward()
            err = max(err, 1.0)
        except RuntimeError:
            pass
        q.put((rank, err, len(red.buckets)))
    except Exception as e:
        q.put((rank, repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


def test_gradient_allreduce_ddp_semantics_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, err, nb in res:
        assert isinstance(err, float), f"rank {rank}: {err}"
        assert err < 1e-6, (rank, err)
        assert nb >= 2
    assert all(p.exitcode == 0 for p in procs)
