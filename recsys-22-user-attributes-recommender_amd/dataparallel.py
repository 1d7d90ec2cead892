"""Data-parallel training (one process per GPU, RCCL over xGMI) with Lightning-DDP gradient semantics.

The reference trains BERT4Rec / KeBERT4Rec data-parallel under PyTorch Lightning's DDP strategy
(configs/ml-20m/unfiltered/bert4rec_config.jsonnet:83-87: `gpus: 8, accelerator: "ddp"`): every rank runs the
whole model on its slice of the batch, computes its OWN masked-mean loss, and the gradients are averaged over
the ranks before each optimizer step.  `GradientAllReduce` reproduces that:

  * the replicated parameters' gradients are all-reduced in fixed-order buckets (~25 MB, reverse registration
    order = the order backward produces them), each launched asynchronously from a post-accumulate-grad hook as
    soon as its last gradient lands -- the RCCL transfer of the output head's gradient overlaps the transformer
    backward -- and buckets are always launched in the same order on every rank (a ready bucket waits for its
    predecessors), as collectives must be;
  * a row-sparse item table (table_grad="sparse": its gradient lives in the step's SparseTablePlan, not in
    .grad) is materialised as the dense (|V|, d) gradient from the plan's deterministic per-row sums and
    all-reduced last; the dense Adam that follows is then exactly DDP's (at C5, |V| ~ 13k: 6.7 MB);
  * finish() waits for every bucket and writes grad / W back into .grad.

For |V| = 10M the table is row-sharded instead (sharded.py): its rows never all-reduce.
Works on any torch.distributed backend ("nccl" = RCCL on ROCm; "gloo" stages device tensors through host memory,
for tests and 1-GPU rehearsals).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import modules as _modules


def _staged(group, t: torch.Tensor) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = params
        self.pending = 0
        self.flat: Optional[torch.Tensor] = None
        self.work = None
        self.host: Optional[torch.Tensor] = None


class GradientAllReduce:
    """Bucketed, backward-overlapped gradient averaging over `group` (DDP semantics)."""

    def __init__(self, module: torch.nn.Module, group=None, bucket_bytes: int = 25 << 20,
                 sharded_table: bool = False):
        """sharded_table: the item table is a row shard (sharded.py) whose gradient reaches its owner through
        the all-to-all exchange; it is left out here entirely (only the replicated parameters are averaged)"""
        self.group = group
        self.world = dist.get_world_size(group)
        self.table = module.model.item_table() if hasattr(module, "model") else None
        params = [p for p in module.parameters() if p.requires_grad]
        if sharded_table and self.table is not None:
            params = [p for p in params if p is not self.table]
        # a row-sparse table arrives through its plan, not through .grad: reduced last (see finish)
        self.sparse_table = (self.table is not None and getattr(module, "table_grad", "dense") == "sparse"
                             and any(p is self.table for p in params))
        ordered = [p for p in reversed(params) if not (self.sparse_table and p is self.table)]
        self.buckets: List[_Bucket] = []
        cur: List[torch.nn.Parameter] = []
        size = 0
        for p in ordered:
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(_Bucket(cur))
                cur, size = [], 0
        if cur:
            self.buckets.append(_Bucket(cur))
        self._bucket_of: Dict[int, _Bucket] = {}
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[id(p)] = b
        self._hooks = [p.register_post_accumulate_grad_hook(self._ready) for b in self.buckets for p in b.params]
        self._next = 0
        self._sync = True
        self._reset()

    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.flat, b.work, b.host = None, None, None
        self._next = 0

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    # ------------------------------------------------------------------------------------------ backward
    @contextlib.contextmanager
    def no_sync(self):
        """gradient accumulation (the reference trainer's accumulate_grad_batches, trainer_builder.py:25): the
        backward passes inside only accumulate into .grad; the next backward outside launches the buckets from
        the accumulated gradients (DDP.no_sync semantics)"""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev
            # (a row-sparse table gradient of these passes cannot be merged with the next one: the next
            # training_step finds its plan holding a gradient -- SparseTablePlan.has_gradient() -- and raises
            # instead of dropping it, modules._TableGradMixin._plan_table)

    def _ready(self, p: torch.nn.Parameter):
        if not self._sync:
            return
        b = self._bucket_of[id(p)]
        if b.pending <= 0 or b.work is not None:
            # a second backward before finish(): its gradient would land after the bucket was reduced and
            # finish() would overwrite the accumulated .grad with the first backward's average
            raise RuntimeError("GradientAllReduce: a gradient hook fired twice before finish(); run the "
                               "accumulation micro-batches inside reducer.no_sync()")
        b.pending -= 1
        if b.pending == 0:
            self._launch_ready()

    def _launch_ready(self, force: bool = False):
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if b.pending > 0 and not force:
                return
            self._launch(b)
            self._next += 1

    def _launch(self, b: _Bucket):
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in b.params]
        b.flat = torch.cat([g.reshape(-1) for g in grads]) if len(grads) > 1 else grads[0].reshape(-1).clone()
        if _staged(self.group, b.flat):
            b.host = b.flat.cpu()
            b.work = dist.all_reduce(b.host, group=self.group, async_op=True)
        else:
            b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)

    # ---------------------------------------------------------------------------------------- after it
    def _table_dense_grad(self) -> Optional[torch.Tensor]:
        """the row-sparse table gradient of this step as a dense (|V|, d) tensor (deterministic ordered row sums)"""
        tg = getattr(self.table, "_asme_table_grad", None)
        plan = tg.plan if tg is not None else None
        dense = torch.zeros_like(self.table)
        if plan is not None:
            U = plan.n_unique()
            dense.index_copy_(0, plan.unique[:U], plan.grad_rows[:U] * plan.grad_scale)
            plan.release()
            tg.plan = None
        return dense

    @torch.no_grad()
    def finish(self):
        """wait for every bucket (launching any whose parameters got no gradient this step), average, write back"""
        self._launch_ready(force=True)
        table_work = None
        if self.sparse_table:
            dense = self._table_dense_grad()
            host = dense.cpu() if _staged(self.group, dense) else None
            table_work = (dense, host, dist.all_reduce(host if host is not None else dense, group=self.group,
                                                       async_op=True))
        inv = 1.0 / self.world
        for b in self.buckets:
            b.work.wait()
            flat = b.flat.copy_(b.host) if b.host is not None else b.flat
            flat.mul_(inv)
            off = 0
            for p in b.params:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n
        if table_work is not None:
            dense, host, work = table_work
            work.wait()
            if host is not None:
                dense.copy_(host)
            dense.mul_(inv)
            self.table.grad = dense
        self._reset()

    def broadcast_parameters(self, module: torch.nn.Module, src: int = 0):
        """make every rank start from rank src's parameters (DDP's constructor broadcast)"""
        with torch.no_grad():
            for p in module.parameters():
                if _staged(self.group, p.data):
                    h = p.data.cpu()
                    dist.broadcast(h, src, group=self.group)
                    p.data.copy_(h)
                else:
                    dist.broadcast(p.data, src, group=self.group)


def train_step(module, optimizer, scheduler, reducer: GradientAllReduce, batch, batch_idx: int = 0) -> torch.Tensor:
    """One data-parallel optimisation step, as Lightning's DDP strategy runs it: this rank's loss on its batch
    slice, backward (gradient buckets all-reduce as they fill), averaged gradients, optimizer + scheduler step."""
    out = module.training_step(batch, batch_idx)
    loss = out["loss"]
    _modules.backward(loss)
    reducer.finish()
    optimizer.step()
    if scheduler is not None:
        scheduler.step()
    optimizer.zero_grad(set_to_none=True)
    return loss
