"""Row-sharded item table across ranks (one process per GPU, RCCL over xGMI) for SASRec-neg training.

The reference trains under Lightning DDP: every rank holds the whole |V| x d table, its dense gradient
is all-reduced and every rank runs dense Adam over all of it.  Here the table is
row-sharded cyclically (global row g -> owner g % W, local row g // W, which spreads Zipf heads) and
only the rows a step touches cross the fabric:

  forward   dedup the step's ids (asme_dedup_ids) -> route unique ids to their owners (all_to_all of
            int64 ids) -> owners bring those rows up to date (lazy exact Adam catch-up) and gather them
            -> all_to_all of the rows back -> the model runs on the compact (U, d) table with remapped ids
  backward  all_to_all of the compact row gradients to the owners (x 1/W: DDP gradient averaging) ->
            owners scatter-add into their step plan -> lazy dense Adam on the shard
  dense params (transformer, position table, LayerNorms) stay replicated; their gradients are
            averaged with one flat all_reduce.
Numerically this is DDP semantics: per-rank mean loss, gradients averaged over ranks, dense Adam over
every row of the (logical) table.

`RowShardExchange` is pure torch.distributed routing (works on gloo/CPU for tests); the data path
around it (dedup, catch-up, gather, scatter, Adam) runs on the gfx950 kernels.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from . import modules as _modules
from . import ops
from .dataparallel import GradientAllReduce
from .modules import (ITEM_SEQ_ENTRY_NAME, NEGATIVE_SAMPLES_ENTRY_NAME, POSITIVE_SAMPLES_ENTRY_NAME,
                      TARGET_ENTRY_NAME, SequenceNextItemPredictionTrainingModule, build_eval_step_return_dict,
                      get_additional_meta_data, get_padding_mask)
from .sequence import InputSequence


def _host_staged(group, t: torch.Tensor) -> bool:
    """gloo has no device all_to_all: device tensors go through host memory (tests / 1-GPU rehearsals of the
    multi-rank path; production runs use the nccl (= RCCL) backend and never stage)"""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None, group=None,
                async_op: bool = False):
    """all_to_all_single; async_op (RCCL): returns the work handle whose wait() makes the CURRENT stream wait for the
    exchange (the host does not block), None when the exchange is already complete (gloo / host-staged)"""
    if _host_staged(group, inp):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return None
    work = dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=async_op)
    if async_op and not out.is_cuda:  # (CPU gloo: complete before the caller reads it)
        work.wait()
        return None
    return work


def _all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None):
    if _host_staged(group, t):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def _broadcast(t: torch.Tensor, src: int, group=None):
    if _host_staged(group, t):
        h = t.cpu()
        dist.broadcast(h, src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src, group=group)


def _all_gather(outs, t: torch.Tensor, group=None):
    if _host_staged(group, t):
        hs = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
        dist.all_gather(hs, t.cpu(), group=group)
        for o, h in zip(outs, hs):
            o.copy_(h)
    else:
        dist.all_gather(outs, t, group=group)


def shard_rows(vocab: int, world: int, rank: int) -> int:
    """number of global rows {rank, rank + W, ...} < vocab owned by `rank`"""
    return max(0, (vocab - rank + world - 1) // world)


@dataclass
class ExchangeState:
    order: torch.Tensor          # send order: the j-th id sent is unique[order[j]] (grouped by owner)
    send_counts: List[int]       # ids sent to each owner
    recv_counts: List[int]       # ids received from each requester
    recv_local: torch.Tensor     # local row ids requested from this rank, grouped by requester
    pos: torch.Tensor            # inverse of order: unique[i] is sent at position pos[i]
    # two-class exchange (request(..., split=...)): the (send, recv) counts of each class; the send order and
    # recv_local are class-major -- [class 0 by owner | class 1 by owner], [class 0 by requester | class 1 by requester]
    classes: Optional[tuple] = None
    work: object = None          # the class-1 rows' reply in flight (reply_rows(..., async_second=True))


class RowShardExchange:
    def __init__(self, vocab: int, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.vocab = vocab
        self.local_rows = shard_rows(vocab, self.world, self.rank)

    def request(self, unique: torch.Tensor, count: Optional[torch.Tensor] = None,
                split: Optional[torch.Tensor] = None) -> ExchangeState:
        """route the requester's unique global ids to their owners (count: int32 (1,) device tensor, only
        unique[:count] are live -- the dedup count, read on the device; the per-owner counts below are the step's
        one host sync).  split (int32 (1,) device tensor): two classes, unique[:split] and the rest, each routed by
        owner in its own exchange (the class-1 rows can then come back while the model already runs)"""
        return self.request_end(self.request_begin(unique, count, split))

    def request_begin(self, unique: torch.Tensor, count: Optional[torch.Tensor] = None,
                      split: Optional[torch.Tensor] = None):
        """first half of request(): owner bucketing and the exchange of the per-owner counts are enqueued and the
        counts are copied to pinned host memory without waiting; request_end() reads them.  Issued a step ahead
        (ShardedSequenceNextItemPredictionTrainingModule.prefetch), the host's read of the split sizes RCCL needs
        no longer drains the GPU's queue."""
        W = self.world
        nbk = 2 * W if split is not None else W
        if unique.is_cuda:  # stable owner bucketing in one counting-sort pass (asme_bucket_by_owner[_split])
            order, send_local, send_counts_t, pos = ops.bucket_by_owner(unique, W, count, split)
        else:
            if count is not None:
                unique = unique[:int(count.item())]
            key = unique % W
            if split is not None:
                key = key + W * (torch.arange(len(unique)) >= int(split.reshape(-1)[0])).to(key.dtype)
            order = torch.argsort(key, stable=True)
            send_counts_t = torch.bincount(key, minlength=nbk).to(torch.int64)
            send_local = (unique.index_select(0, order) // W).to(torch.int32)
            pos = torch.empty_like(order)
            pos[order] = torch.arange(len(order), dtype=order.dtype)
        if split is not None:
            # per destination rank the pair (class-0 count, class-1 count): one (W, 2) exchange
            sendm = send_counts_t.view(2, W).t().contiguous()
            recvm = torch.empty_like(sendm)
            _all_to_all(recvm, sendm, group=self.group)
            counts = torch.stack([send_counts_t, recvm.t().reshape(-1)])  # both class-major (2 W)
        else:
            recv_counts_t = torch.empty_like(send_counts_t)
            _all_to_all(recv_counts_t, send_counts_t, group=self.group)
            counts = torch.stack([send_counts_t, recv_counts_t])
        event = None
        if counts.is_cuda:
            host = torch.empty(counts.shape, dtype=counts.dtype, pin_memory=True)
            host.copy_(counts, non_blocking=True)
            event = torch.cuda.Event()
            event.record()
        else:
            host = counts
        return (order, send_local, pos, host, event, unique.device, split is not None)

    def request_end(self, pending) -> ExchangeState:
        order, send_local, pos, host, event, dev, two = pending
        if event is not None:
            event.synchronize()  # the step's one host sync
        W = self.world
        # owner-local rows cross the fabric as int32 (a shard holds < 2^31 rows); widened once on arrival for the
        # gather / dedup kernels, which take int64 row ids
        if not two:
            sc, rc = host[0].tolist(), host[1].tolist()
            recv32 = torch.empty(sum(rc), dtype=torch.int32, device=dev)
            _all_to_all(recv32, send_local[:sum(sc)], rc, sc, group=self.group)
            return ExchangeState(order[:sum(sc)], sc, rc, recv32.to(torch.int64), pos)
        s_all, r_all = host[0].tolist(), host[1].tolist()
        sc0, sc1, rc0, rc1 = s_all[:W], s_all[W:], r_all[:W], r_all[W:]
        n0 = sum(sc0)
        recv32 = torch.empty(sum(rc0) + sum(rc1), dtype=torch.int32, device=dev)
        _all_to_all(recv32[:sum(rc0)], send_local[:n0], rc0, sc0, group=self.group)
        _all_to_all(recv32[sum(rc0):], send_local[n0:n0 + sum(sc1)], rc1, sc1, group=self.group)
        sc = [a + b for a, b in zip(sc0, sc1)]
        rc = [a + b for a, b in zip(rc0, rc1)]
        return ExchangeState(order[:n0 + sum(sc1)], sc, rc, recv32.to(torch.int64), pos, classes=(sc0, sc1, rc0, rc1))

    def reply_rows(self, st: ExchangeState, rows: torch.Tensor, async_second: bool = False) -> torch.Tensor:
        """owners' rows (aligned with st.recv_local) -> the requester's rows in SEND order: row j belongs to
        unique[st.order[j]] (unique id i is row st.pos[i]; callers remap ids instead of permuting rows).
        A two-class state sends the class-0 rows, then the class-1 rows -- with async_second in flight on RCCL's
        stream when this returns (st.work: wait() on it before reading rows past the class-0 block)"""
        if self.world == 1:  # the rank's own rows in request order: no copy
            return rows.detach().contiguous()
        U = len(st.order)
        got = torch.empty(U, rows.shape[1], dtype=rows.dtype, device=rows.device)
        rows = rows.contiguous()
        if st.classes is None:
            _all_to_all(got, rows, st.send_counts, st.recv_counts, group=self.group)
            return got
        sc0, sc1, rc0, rc1 = st.classes
        n0, r0 = sum(sc0), sum(rc0)
        _all_to_all(got[:n0], rows[:r0], sc0, rc0, group=self.group)
        st.work = _all_to_all(got[n0:], rows[r0:], sc1, rc1, group=self.group, async_op=async_second)
        return got

    def push_grads(self, st: ExchangeState, grad_send: torch.Tensor) -> torch.Tensor:
        """requester's gradient rows in send order (aligned with reply_rows) -> owners, aligned with recv_local"""
        if self.world == 1:
            return grad_send.contiguous()
        recv = torch.empty(len(st.recv_local), grad_send.shape[1], dtype=grad_send.dtype, device=grad_send.device)
        grad_send = grad_send.contiguous()
        if st.classes is None:
            _all_to_all(recv, grad_send, st.recv_counts, st.send_counts, group=self.group)
            return recv
        sc0, sc1, rc0, rc1 = st.classes
        n0, r0 = sum(sc0), sum(rc0)
        _all_to_all(recv[:r0], grad_send[:n0], rc0, sc0, group=self.group)
        _all_to_all(recv[r0:], grad_send[n0:], rc1, sc1, group=self.group)
        return recv


class ShardedSequenceNextItemPredictionTrainingModule(SequenceNextItemPredictionTrainingModule):
    """sasrec-neg training with the item table row-sharded over the process group.

    Build the model with item_vocab_size = shard_rows(V, W, rank) (the local shard); `vocab` is the
    global |V|.  Call `after_backward()` between loss.backward() and optimizer.step() (train_step in
    this module does it)."""

    def __init__(self, model, item_tokenizer, metrics, vocab: int, learning_rate: float = 0.001,
                 beta_1: float = 0.99, beta_2: float = 0.998, weight_decay: float = 1e-3, loss_function=None,
                 group=None, overlap_negatives: bool = False):
        """overlap_negatives (W > 1): the rows only the sampled head reads -- ids that occur among the negatives but
        not in the sequence or the positives, ~half the step's distinct rows -- come back in a second all-to-all
        that runs on RCCL's stream while the embedding and the transformer compute; the head waits for it.  Their
        gradients go back in a second all-to-all too.  Same owner plan (one dedup, one lazy-Adam staging, one
        ordered reduction over every requester's rows), DDP semantics unchanged."""
        super().__init__(model, item_tokenizer, metrics, learning_rate, beta_1, beta_2, weight_decay,
                         loss_function, table_grad="sparse")
        self.overlap_negatives = overlap_negatives
        self.exchange = RowShardExchange(vocab, group)
        self.vocab = vocab
        self.group = group
        shard = model.item_table()
        if shard.shape[0] != self.exchange.local_rows:
            raise ValueError(f"model item table has {shard.shape[0]} rows, shard needs {self.exchange.local_rows}")
        self._req_map: Optional[torch.Tensor] = None
        self._own_map: Optional[torch.Tensor] = None
        self._pending = None
        self._prefetched = None  # (caller's id tensors, normalised id sets, requester plan, request_begin state)
        self.prefetch_hits = 0   # training steps that consumed a prefetch (tests assert the overlap really ran)
        # the replicated parameters average through the bucketed, backward-overlapped all-reduce (DDP semantics);
        # the shard is excluded (its rows travel to their owners in after_backward)
        self.reducer = (GradientAllReduce(self, group, sharded_table=True)
                        if self.exchange.world > 1 else None)

    def broadcast_dense_parameters(self, src: int = 0):
        """make the replicated (non-table) parameters identical on every rank"""
        shard = self.model.item_table()
        for p in self.model.parameters():
            if p is not shard:
                _broadcast(p.data, src, group=self.group)

    def _maps(self, dev):
        if self._req_map is None:
            self._req_map = torch.full((self.vocab,), -1, dtype=torch.int32, device=dev)
            self._own_map = torch.full((max(1, self.exchange.local_rows),), -1, dtype=torch.int32, device=dev)

    _ID_KEYS = (ITEM_SEQ_ENTRY_NAME, POSITIVE_SAMPLES_ENTRY_NAME, NEGATIVE_SAMPLES_ENTRY_NAME)

    def prefetch(self, batch):
        """Start the routing of the NEXT step's ids now: its dedup, owner bucketing and the exchange of the
        per-owner counts are enqueued, and the counts copied to the host asynchronously.  Called after the
        current step's forward (sharded.train_step's next_batch), the host reads those split sizes while the GPU
        still runs the current backward, instead of draining the queue at the next step's start.

        Contract (collective): every rank calls it at the same point, and the NEXT training_step on every rank
        receives the very same id tensor objects (int32 or int64, any layout), unmodified in between.  That
        step always consumes the prefetch -- so every rank runs the same collective sequence -- and raises if its
        batch is not the prefetched one (a silent re-route on one rank only would misalign the collectives)."""
        self.cancel_prefetch()
        originals = tuple(batch[k] for k in self._ID_KEYS)
        batch = self._ids_i64(batch, self._ID_KEYS)
        id_sets = [batch[k] for k in self._ID_KEYS]
        self._maps(self.model.item_table().device)
        req = ops.SparseTablePlan.for_ids(self.vocab, id_sets, self._req_map)
        self._prefetched = (originals, id_sets, req,
                            self.exchange.request_begin(req.unique, req.count, self._split(req, id_sets)))

    def _split(self, req, id_sets) -> Optional[torch.Tensor]:
        """overlap_negatives: the requester's class boundary (int32 (1,) on the device) -- the dedup numbers the unique
        ids in first-occurrence order over [sequence, positives, negatives], so the ids the sequence or the positives
        hold are exactly the slots below max(their slots) + 1 and every slot past it is a negative-only row"""
        if not self.overlap_negatives or self.exchange.world == 1 or len(id_sets) != 3:
            return None
        n_a = id_sets[0].numel() + id_sets[1].numel()
        if n_a == 0:
            return torch.zeros(1, dtype=torch.int32, device=req.unique.device)
        return (req._flat_inverse[:n_a].max() + 1).to(torch.int32).reshape(1)

    def cancel_prefetch(self):
        """drop a prefetched request that will not be used (its counts exchange is complete on every rank);
        collective in effect: every rank must cancel the same prefetch"""
        if self._prefetched is not None:
            self._prefetched[2].release()
            self._prefetched = None

    def _fetch(self, id_sets, train: bool, originals=None):
        """dedup the ids of `id_sets`, route them to their owners, gather the (caught-up) rows and return
        (exchange state, owner plan or None, compact rows in send order, each id set remapped to them).
        originals: the caller's id tensors before normalisation (a training step): a pending prefetch is
        consumed, and must be of exactly these tensors"""
        shard = self.model.item_table()
        self._maps(shard.device)
        pre = None
        if self._prefetched is not None and originals is None:
            self.cancel_prefetch()  # an evaluation between prefetch and step: dropped on every rank (collective)
        elif self._prefetched is not None:
            pre, self._prefetched = self._prefetched, None
            if len(pre[0]) != len(originals) or any(a is not b for a, b in zip(pre[0], originals)):
                pre[2].release()
                raise RuntimeError("sharded training_step received a batch other than the one passed to prefetch(); "
                                   "pass the prefetched batch's tensors (or call cancel_prefetch() on every rank)")
        if pre is not None:
            # 1.-2. dedup and the counts exchange were issued a step ahead (prefetch); the prefetch normalised
            # the same tensors, so the plan's registered id sets are the ones this step reads
            id_sets[:] = pre[1]
            req = pre[2]
            st = self.exchange.request_end(pre[3])
            self.prefetch_hits += 1
        else:
            # 1. requester: dedup every id of the step
            req = ops.SparseTablePlan.for_ids(self.vocab, id_sets, self._req_map)
            # 2. route ids to owners (the dedup count stays on the device); owners bring their rows up to date
            # (lazy Adam: staged in slot order, or caught up in the table) and gather them
            st = self.exchange.request(req.unique, req.count, self._split(req, id_sets) if train else None)
        own = None
        src, src_ids = shard.detach(), st.recv_local
        if train:
            if self.exchange.world == 1:
                # one rank: the requests are the requester's unique ids -- distinct, no owner dedup / CSR
                own = ops.SparseTablePlan.distinct(shard, st.recv_local, self._own_map)
            else:
                own = ops.SparseTablePlan(shard, [st.recv_local], self._own_map)
                own.grad_scale = 1.0 / self.exchange.world  # DDP averaging, applied in the ordered row sums
            src, src_ids = own.gather_source(shard.detach(), st.recv_local)
        with torch.no_grad():
            if src_ids is None:  # the staged rows are the requested rows, in request order
                rows = src[:len(st.recv_local)]
            else:
                rows = ops.gather_rows(src_ids, src) if len(st.recv_local) else shard.new_empty(0, shard.shape[1])
        # the compact table stays in send order; the ids are remapped to it (no row permutation).  Two classes: the
        # negative-only rows' reply stays in flight (st.work), past the class-0 block the model reads first
        compact = self.exchange.reply_rows(st, rows, async_second=True)
        inv = [st.pos.index_select(0, req.inverse_of(x).reshape(-1)).view(x.shape) for x in id_sets]
        req.release()
        return st, own, compact, inv

    def training_step(self, batch, batch_idx):
        self._catalog_planes.clear()  # (the evaluation's shard planes are stale from here on)
        originals = tuple(batch[k] for k in self._ID_KEYS)
        batch = self._ids_i64(batch, self._ID_KEYS)
        id_sets = [batch[k] for k in self._ID_KEYS]
        st, own, compact, (inv_seq, inv_pos, inv_neg) = self._fetch(id_sets, train=True, originals=originals)
        input_seq = id_sets[0]
        compact.requires_grad_(True)
        U = compact.shape[0]
        # its gradient: the heads' contributions summed per compact row in a fixed order (no float atomics, no zero fill)
        cplan = ops.SparseTablePlan.identity(U, [inv_seq, inv_pos, inv_neg], compact.shape[1])
        compact._asme_table_grad = ops.TableGrad()
        compact._asme_table_grad.plan = cplan
        # 3. the model runs on the compact table
        emb = self.model._sequence_embedding_layer.item_embedding_layer
        meta = get_additional_meta_data(self.model, batch)
        meta["positive_samples"], meta["negative_samples"] = inv_pos, inv_neg
        padding_mask = get_padding_mask(input_seq, self.item_tokenizer)
        emb._table_override = compact
        wait, pending = None, []
        if st.work is not None:  # the negative-only rows are still arriving: the sampled head waits for them
            pending.append(st.work)
            st.work = None

            def _wait(module, args):  # (returns None: the head's inputs unchanged)
                while pending:
                    pending.pop().wait()
            wait = self.model._projection_layer.register_forward_pre_hook(_wait)
        try:
            pos_logits, neg_logits = self.model(InputSequence(inv_seq, padding_mask, meta))
        finally:
            emb._table_override = None
            if wait is not None:
                wait.remove()
            while pending:  # a forward that never reached the head (or raised): the exchange still completes here
                pending.pop().wait()
        loss = self.loss_function(pos_logits, neg_logits, mask=padding_mask)
        self._pending = (st, own, compact, cplan)
        return {"loss": loss}

    @torch.no_grad()
    def after_backward(self):
        """average the replicated gradients (their buckets were launched during the backward) and route the
        compact table gradient to the owners.  Collective order, identical on every rank: the bucket all-reduces
        (hooks, then finish's forced launches), then the gradient all-to-all."""
        st, own, compact, cplan = self._pending
        self._pending = None
        if self.reducer is not None:
            self.reducer.finish()
        shard = self.model.item_table()
        if self.exchange.world == 1 and own is not None and own._distinct and compact.grad is None \
                and cplan.has_gradient() and cplan._grad_rows is None:
            # one rank: compact row s IS the owner's slot s, so the owner reduces the requester's occurrences
            # directly and applies the step in the same pass (asme_table_grad_reduce_apply) -- no compact gradient
            # rows, no exchange
            own.adopt_contributions(cplan)
            shard._asme_table_grad.plan = own
            return
        g = cplan.grad_rows[:compact.shape[0]]
        if compact.grad is not None:  # a head without the plan path returned a dense gradient
            g = g + compact.grad
        recv = self.exchange.push_grads(st, g)
        cplan.release()
        if len(st.recv_local):
            own.add_rows(st.recv_local, recv)  # ordered per-row sums x 1/W (deterministic)
        shard._asme_table_grad.plan = own


    # ---------------------------------------------------------------- evaluation on the sharded table
    @torch.no_grad()
    def catalog_ranks(self, batch) -> torch.Tensor:
        """1-based full-catalogue rank of every sequence's target over the GLOBAL item table: the input rows
        come from their owners, each rank scores every rank's queries against its own shard
        (sharded.catalog_ranks).  Collective: every rank must call it with the same batch size."""
        self._flush_table()  # the shard's deferred Adam rows, before anyone reads them
        batch = self._ids_i64(batch, (ITEM_SEQ_ENTRY_NAME, TARGET_ENTRY_NAME))
        input_seq, targets = batch[ITEM_SEQ_ENTRY_NAME], batch[TARGET_ENTRY_NAME]
        _, _, compact, (inv_seq,) = self._fetch([input_seq], train=False)
        compact._asme_table_grad = ops.TableGrad()  # no plan: the gather kernels read it like any table
        emb = self.model._sequence_embedding_layer.item_embedding_layer
        meta = get_additional_meta_data(self.model, batch)
        padding_mask = get_padding_mask(input_seq, self.item_tokenizer)
        emb._table_override = compact
        try:
            q = self.model.catalog_query(InputSequence(inv_seq, padding_mask, meta))
        finally:
            emb._table_override = None
        if q is None or q[2] is not None:
            raise NotImplementedError("sharded evaluation needs the tied dot-product projection")
        shard = self.model.item_table().detach()
        return catalog_ranks(self.exchange, q[0], targets, shard, planes=self._catalog_planes.get(shard))

    def validation_step(self, batch, batch_idx):
        """NDCG / recall / MRR of the sharded model, identical to the unsharded model's (ranks over all |V|)"""
        if self.metrics is None or not hasattr(self.metrics, "update_ranks"):
            raise NotImplementedError("sharded validation needs a rank-based metrics container")
        targets = batch[TARGET_ENTRY_NAME]
        if targets.dim() != 1:
            raise NotImplementedError("sharded validation takes one target per sequence")
        self.metrics.update_ranks(self.catalog_ranks(batch))
        return build_eval_step_return_dict(batch[ITEM_SEQ_ENTRY_NAME], None, targets)

    def test_step(self, batch, batch_idx):
        return self.validation_step(batch, batch_idx)

    def predict_step(self, batch, batch_idx, dataloader_idx=None):
        raise NotImplementedError("predict_step would score every item of the global table on one rank; use "
                                  "catalog_ranks / sharded.catalog_topk")


def train_step(module, optimizer, batch, batch_idx: int = 0, next_batch=None):
    """one sharded training step; with next_batch (the batch the following call will receive) the next step's id
    routing is started after this step's forward (module.prefetch), overlapping its host sync with the backward"""
    out = module.training_step(batch, batch_idx)
    if next_batch is not None:
        module.prefetch(next_batch)
    loss = out["loss"]
    _modules.backward(loss)
    module.after_backward()
    optimizer.step()
    optimizer.zero_grad(set_to_none=True)
    return loss


# ------------------------------------------------------------------------------------ sharded evaluation
def _gather_queries(x: torch.Tensor, group) -> torch.Tensor:
    W = dist.get_world_size(group)
    out = [torch.empty_like(x) for _ in range(W)]
    _all_gather(out, x.contiguous(), group=group)
    return torch.cat(out, 0)


def catalog_ranks(exchange: RowShardExchange, hidden: torch.Tensor, targets: torch.Tensor,
                  table_shard: torch.Tensor, planes: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Full-catalogue rank of every query's target with the item table row-sharded.

    Every rank holds its own queries (hidden (n, d), targets (n,), n equal on all ranks).  The target rows
    come from their owners (one all_to_all pair), the target scores are computed once by the same MFMA
    sequence the shard scans use; every rank then counts, for the queries of ALL ranks, the items of ITS
    shard that rank above the target (asme_catalog_count_above, no logits); one all_reduce(sum) of the
    int32 counts gives the global ranks.  The table shard must be up to date (flush the lazy Adam first); `planes`:
    ops.catalog_planes(table_shard) made earlier (a validation pass splits its shard once)."""
    group, W, rank = exchange.group, exchange.world, exchange.rank
    uniq, inv = torch.unique(targets, return_inverse=True)
    st = exchange.request(uniq)
    got = exchange.reply_rows(st, table_shard.index_select(0, st.recv_local))  # send order
    tscore = ops.catalog_target_scores(hidden, got.index_select(0, st.pos.index_select(0, inv)))
    h_all = _gather_queries(hidden, group)
    t_all = _gather_queries(targets.to(torch.int64), group)
    s_all = _gather_queries(tscore, group)
    counts = ops.catalog_count_above(h_all, table_shard, t_all, s_all, W, rank, planes=planes)
    _all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    n = hidden.shape[0]
    return counts[rank * n:(rank + 1) * n].to(torch.int64) + 1


def catalog_topk(exchange: RowShardExchange, hidden: torch.Tensor, table_shard: torch.Tensor, k: int):
    """Global top-k (score desc, item id asc) over the row-sharded table: every rank scores all ranks'
    queries against its shard (asme_catalog_topk with global ids), the (k) candidates per shard are
    all-gathered and merged."""
    group, W, rank = exchange.group, exchange.world, exchange.rank
    n = hidden.shape[0]
    h_all = _gather_queries(hidden, group)
    v, i = ops.catalog_topk(h_all, table_shard, k, id_stride=W, id_offset=rank)
    vs = [torch.empty_like(v) for _ in range(W)]
    is_ = [torch.empty_like(i) for _ in range(W)]
    _all_gather(vs, v, group=group)
    _all_gather(is_, i, group=group)
    cand_v = torch.cat([x[rank * n:(rank + 1) * n] for x in vs], 1)
    cand_i = torch.cat([x[rank * n:(rank + 1) * n] for x in is_], 1)
    # (score desc, id asc): sort by id, then stably by score
    o1 = torch.argsort(cand_i, dim=1, stable=True)
    cand_v, cand_i = cand_v.gather(1, o1), cand_i.gather(1, o1)
    o2 = torch.argsort(-cand_v, dim=1, stable=True)
    return cand_v.gather(1, o2)[:, :k], cand_i.gather(1, o2)[:, :k]
