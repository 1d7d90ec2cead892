"""Full-catalogue evaluation without materialised logits (csrc/catalog.hip): sharding arithmetic,
the module's fused validation path, and the RCCL sharded-eval entry points on a 1-rank group."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_catalog_shard_counts_sum_to_full_rank(asme, dev):
    """ranks over a cyclically row-sharded table = ranks over the whole table."""
    torch.manual_seed(0)
    nq, V, d, W = 200, 5003, 64, 3
    H = torch.randn(nq, d, device=dev)
    E = torch.randn(V, d, device=dev)
    targets = torch.randint(0, V, (nq,), device=dev)
    full = asme.ops.catalog_rank(H, E, targets)
    tscore = asme.ops.catalog_target_scores(H, E.index_select(0, targets))
    total = torch.zeros(nq, dtype=torch.int64, device=dev)
    for r in range(W):
        shard = E[r::W].contiguous()
        total += asme.ops.catalog_count_above(H, shard, targets, tscore, W, r).to(torch.int64)
    assert torch.equal(total + 1, full)
    # top-k from per-shard candidates with global ids
    k = 10
    v_full, i_full = asme.ops.catalog_topk(H, E, k)
    cand_v, cand_i = [], []
    for r in range(W):
        v, i = asme.ops.catalog_topk(H, E[r::W].contiguous(), k, id_stride=W, id_offset=r)
        cand_v.append(v)
        cand_i.append(i)
    cv, ci = torch.cat(cand_v, 1), torch.cat(cand_i, 1)
    o = torch.argsort(-cv, dim=1, stable=True)
    assert torch.equal(ci.gather(1, o)[:, :k], i_full)


def test_module_fused_eval_matches_materialised(asme, dev):
    """SASRec validation: NDCG/recall/MRR from asme_catalog_rank == from the (B, |V|) predictions."""
    from helpers import build_model, load, state_dict
    z = load("sasrec_neg")
    V = int(z["cfg"][5])
    model = build_model(asme, "sasrec_neg", z)
    model.load_state_dict(state_dict(z))
    model.to(dev).eval()
    tok = asme.tokenization.Tokenizer(V - 3)
    seq = torch.from_numpy(z["seq"]).to(dev)
    targets = torch.from_numpy(z["pos"]).to(dev)[:, -1].contiguous()
    batch = {"item": seq, "item.target": targets}
    res = []
    for fused in (False, True):
        metrics = asme.metrics.RankingMetricsContainer([asme.metrics.NormalizedDiscountedCumulativeGainMetric(5),
                                                        asme.metrics.RecallMetric(5), asme.metrics.MRRMetric(5)])
        module = asme.SequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=metrics,
                                                                fused_eval=fused)
        with torch.no_grad():
            out = module.validation_step(batch, 0)
        assert (out["predictions"] is None) == fused
        res.append({k: float(v) for k, v in metrics.compute().items()})
    assert res[0].keys() == res[1].keys()
    for k in res[0]:
        assert abs(res[0][k] - res[1][k]) < 1e-6, k


def test_sharded_eval_single_rank(asme, dev):
    import torch.distributed as dist
    torch.manual_seed(1)
    nq, V, d = 96, 4000, 128
    H = torch.randn(nq, d, device=dev)
    E = torch.randn(V, d, device=dev)
    targets = torch.randint(0, V, (nq,), device=dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    fresh = not dist.is_initialized()
    if fresh:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        ex = asme.sharded.RowShardExchange(V)
        ranks = asme.sharded.catalog_ranks(ex, H, targets, E)
        assert torch.equal(ranks, asme.ops.catalog_rank(H, E, targets))
        v, i = asme.sharded.catalog_topk(ex, H, E, 8)
        v0, i0 = asme.ops.catalog_topk(H, E, 8)
        assert torch.equal(i, i0) and torch.equal(v, v0)
    finally:
        if fresh:
            dist.destroy_process_group()


def test_catalog_rank_and_topk_at_ten_million_items(asme, dev):
    """SURVEY §8f row 1 at its full size: ranks and top-k of 512 queries over |V| = 10,000,003 items, d = 128
    (BASELINE C4's catalogue), without materialising the (512, 10M) scores, against a chunked float64 torch
    reference on the same device.  The kernel scores in fp32, so a target's rank is exact up to the items whose
    float64 score lies within the fp32 error band of the target's (eps = 2e-6 of sum |h_k e_k| per score, both
    sides): 1 + #{s > t + eps} <= rank <= 1 + #{s > t - eps} (minus the target itself).  At 10M items the band holds
    up to a few hundred items around the median score (~4M items per unit of score), none near the top."""
    torch.manual_seed(10)
    nq, V, d, k = 512, 10_000_003, 128, 10
    E = torch.randn(V, d, device=dev) / d ** 0.5
    H = torch.randn(nq, d, device=dev)
    targets = torch.randint(0, V, (nq,), device=dev)
    # a few targets near the top of their rows, so the ranks are not all ~V/2
    top_ids = asme.ops.catalog_topk(H[:8], E, 1)[1][:, 0]
    targets[:8] = top_ids
    ranks = asme.ops.catalog_rank(H, E, targets)
    vals, idx = asme.ops.catalog_topk(H, E, k)
    torch.cuda.synchronize()
    H64 = H.double()
    Et = E.index_select(0, targets).double()
    t64 = (H64 * Et).sum(1)
    rel = 2e-6
    eps_t = rel * (H64.abs() * Et.abs()).sum(1)
    A64 = H64.abs()
    lo = torch.zeros(nq, dtype=torch.int64, device=dev)
    hi = torch.zeros(nq, dtype=torch.int64, device=dev)
    best_v = torch.full((nq, k), -float("inf"), dtype=torch.float64, device=dev)
    best_e = torch.zeros((nq, k), dtype=torch.float64, device=dev)
    chunk = 1 << 20
    for c0 in range(0, V, chunk):
        Ec = E[c0:c0 + chunk].double()
        s = H64 @ Ec.t()
        eps = rel * (A64 @ Ec.abs().t()) + eps_t[:, None]
        lo += (s > t64[:, None] + eps).sum(1)
        hi += (s > t64[:, None] - eps).sum(1)
        v, j = torch.topk(s, k, dim=1)
        cand_v, cand_e = torch.cat([best_v, v], 1), torch.cat([best_e, eps.gather(1, j)], 1)
        best_v, o = torch.topk(cand_v, k, dim=1)
        best_e = cand_e.gather(1, o)
        del s, eps, Ec
    hi -= 1  # the target's own score is inside its band
    assert bool(((1 + lo) <= ranks).all()) and bool((ranks <= (1 + hi)).all())
    assert int((hi - lo).max()) <= 2000, int((hi - lo).max())
    assert int(ranks[:8].max()) <= 1 + int((hi - lo)[:8].max())  # the top-1 targets rank (near) first
    # top-k: each returned item's float64 score matches its value and belongs to the float64 top-k (up to the band)
    Ei = E.index_select(0, idx.reshape(-1)).double().view(nq, k, d)
    s_idx = (H64[:, None, :] * Ei).sum(2)
    e_idx = rel * (A64[:, None, :] * Ei.abs()).sum(2)
    assert bool(((s_idx - vals.double()).abs() <= e_idx).all())
    assert bool((vals[:, :-1] >= vals[:, 1:]).all())
    assert bool((s_idx >= best_v[:, -1:] - e_idx - best_e[:, -1:]).all())
    assert bool((idx >= 0).all()) and bool((idx < V).all())
    assert all(len(set(r)) == k for r in idx.tolist())


@pytest.mark.parametrize("nq,V,d,with_bias", [(300, 5003, 128, True), (1024, 27003, 128, False), (37, 999, 64, True)])
def test_catalog_rank_equals_rank_of_materialised_scores(asme, dev, nq, V, d, with_bias):
    """asme_catalog_rank_x6 (bf16x6 scores streamed, never stored) == the rank read off asme_logits' materialised
    scores (the same products): 1 + #{s > s_t} + #{s == s_t, id < t}, exactly; a catalogue split once
    (ops.catalog_planes) and reused gives the same ranks"""
    torch.manual_seed(nq + V)
    H = torch.randn(nq, d, device=dev)
    E = torch.randn(V, d, device=dev) / d ** 0.5
    b = torch.randn(V, device=dev) if with_bias else None
    targets = torch.randint(0, V, (nq,), device=dev)
    ranks = asme.ops.catalog_rank(H, E, targets, b)
    with torch.no_grad():
        S = asme.ops.logits(H, E, b)
    st = S.gather(1, targets[:, None])
    ids = torch.arange(V, device=dev)[None, :]
    want = 1 + ((S > st) | ((S == st) & (ids < targets[:, None]))).sum(1)
    assert torch.equal(ranks, want)
    planes = asme.ops.catalog_planes(E)
    assert torch.equal(asme.ops.catalog_rank(H, E, targets, b, planes=planes), want)
    # ties: duplicated item rows score identically; the lower id ranks first
    E2 = E.clone()
    E2[1::2] = E2[0::2][: E2[1::2].shape[0]]
    r2 = asme.ops.catalog_rank(H, E2, targets, None)
    S2 = asme.ops.logits(H, E2, None)
    st2 = S2.gather(1, targets[:, None])
    want2 = 1 + ((S2 > st2) | ((S2 == st2) & (ids < targets[:, None]))).sum(1)
    assert torch.equal(r2, want2)


@pytest.mark.parametrize("with_bias", [False, True])
def test_catalog_rank_far_ties_and_invalid_targets(asme, dev, with_bias):
    """Exact ties on the branch-free clean path (logits.hip M_RANK: a 32-row sub-tile holding neither the target's
    row nor its lower-id boundary compares with s_t, or with the float just below s_t): every target's row is copied
    5,000 rows above it and 6,000 rows below it -- other sub-tiles and chunks, one tie of a higher and one of a lower
    id -- for positive and negative target scores (queries h and -h).  The ranks equal those read off the
    materialised scores, unsharded (asme_catalog_rank_x6) and through the sharded count (asme_catalog_count_above_x6
    over W = 3 cyclic shards, id_stride 3, id_offset r).  Targets -1 and V rank as item 0 (the score gather clamps
    them to item 0, and so does the rank test)."""
    torch.manual_seed(17 + with_bias)
    V, d, nq = 27003, 128, 512
    H = torch.randn(nq // 2, d, device=dev)
    H = torch.cat([H, -H])
    E = torch.randn(V, d, device=dev) / d ** 0.5
    b = torch.randn(V, device=dev) if with_bias else None
    targets = torch.randint(10000, 12000, (nq,), device=dev)
    E2, b2 = E.clone(), (b.clone() if b is not None else None)
    for off in (5000, -6000):
        E2[targets + off] = E[targets]
        if b2 is not None:
            b2[targets + off] = b[targets]
    S = asme.ops.logits(H, E2, b2)
    ids = torch.arange(V, device=dev)[None, :]

    def want_of(tg):
        st = S.gather(1, tg[:, None])
        return 1 + ((S > st) | ((S == st) & (ids < tg[:, None]))).sum(1)

    want = want_of(targets)
    st = S.gather(1, targets[:, None])[:, 0]
    assert bool((st > 0).any()) and bool((st < 0).any())
    ties = ((S == st[:, None]).sum(1) - 1)
    assert int((ties >= 2).sum()) >= nq * 0.9  # the copies really tie (up and down)
    assert torch.equal(asme.ops.catalog_rank(H, E2, targets, b2), want)
    # sharded: W = 3 cyclic shards (row g on rank g % 3), counts summed, target scores from the target rows
    tscore = asme.ops.catalog_target_scores(H, E2.index_select(0, targets),
                                             b2.index_select(0, targets) if b2 is not None else None)
    total = torch.zeros(nq, dtype=torch.int64, device=dev)
    for r in range(3):
        shard = E2[r::3].contiguous()
        bs = b2[r::3].contiguous() if b2 is not None else None
        total += asme.ops.catalog_count_above(H, shard, targets, tscore, 3, r, bs).to(torch.int64)
    assert torch.equal(total + 1, want)
    # invalid targets: ranked as item 0
    bad = targets.clone()
    bad[:16] = -1
    bad[16:32] = V
    got = asme.ops.catalog_rank(H, E2, bad, b2)
    fix = bad.clone()
    fix[:32] = 0
    assert torch.equal(got, want_of(fix))


def test_catalog_planes_cache_follows_every_table_write(asme, dev):
    """ops.CatalogPlanes reuses the split while the catalogue is unchanged and re-splits after any write: a torch
    in-place op (version counter), a FusedAdam step (kernels writing behind the counter); the module's validation
    ranks after a training step equal a fresh split's."""
    ops = asme.ops
    torch.manual_seed(3)
    E = torch.randn(5003, 64, device=dev)
    c = ops.CatalogPlanes()
    p1 = c.get(E)
    assert c.get(E) is p1 and c.get(E.detach()) is p1  # (detach shares storage and version counter)
    assert torch.equal(p1, ops.catalog_planes(E))
    E.add_(1e-3)
    p2 = c.get(E)
    assert p2 is not p1 and torch.equal(p2, ops.catalog_planes(E))
    ops.note_param_write()
    assert c.get(E) is not p2
    # a table _f32 has to copy (not contiguous) is never cached
    En = torch.randn(5003, 128, device=dev)[:, :64]
    assert c.get(En) is not c.get(En)

    from helpers import build_model, load, state_dict
    z = load("sasrec_neg")
    V = int(z["cfg"][5])
    model = build_model(asme, "sasrec_neg", z)
    model.load_state_dict(state_dict(z))
    model.to(dev)
    tok = asme.tokenization.Tokenizer(V - 3)
    seq = torch.from_numpy(z["seq"]).to(dev)
    pos = torch.from_numpy(z["pos"]).to(dev)
    neg = torch.from_numpy(z["neg"]).to(dev)
    eval_batch = {"item": seq, "item.target": pos[:, -1].contiguous()}
    module = asme.SequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=None,
                                                            fused_eval=True)
    opt = module.configure_optimizers()
    module.eval()
    with torch.no_grad():
        r0 = module.catalog_ranks(eval_batch)
        planes = module._catalog_planes._planes
        assert torch.equal(module.catalog_ranks(eval_batch), r0) and module._catalog_planes._planes is planes
    module.train()
    out = module.training_step({"item": seq, "positive_samples": pos, "negative_samples": neg}, 0)
    asme.modules.backward(out["loss"])
    opt.step()
    opt.zero_grad()
    module.eval()
    with torch.no_grad():
        r1 = module.catalog_ranks(eval_batch)
        table = model.item_table()
        h, _, bias = model.catalog_query(asme.sequence.InputSequence(
            seq, asme.modules.get_padding_mask(seq, tok), {}))
        fresh = ops.catalog_rank(h, table, eval_batch["item.target"], bias)
    assert module._catalog_planes._planes is not planes
    assert torch.equal(r1, fresh)
    # a flush with nothing deferred writes nothing and keeps the split; a catch-up that replays rows drops it
    kept = module._catalog_planes.get(table)
    opt.flush()
    assert module._catalog_planes.get(table) is kept
    lazy = table._asme_table_grad.lazy
    lazy.record(lazy.step + 1, 1e-3, 0.9, 0.998, 1e-8, 1e-3)  # a zero-gradient step, replayed by the next flush
    opt.flush()  # (LazyTableState.catch_up writes every row behind torch's version counter)
    assert module._catalog_planes.get(table) is not kept
