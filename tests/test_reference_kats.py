"""CPU: known-answer values from the reference's own test-suite, applied to the oracle and to the
product's host-side metric logic.

Values are the assertion values of /root/reference/tests/test_ndcg.py (EPSILON = 10e-4 as in
tests/util_test_metric.py:11); they pin calc_ndcg / calc_dcg semantics incl. IDCG truncation.
"""
import numpy as np
import pytest
import torch

from oracle import asme_oracle as O

EPS = 10e-4
SINGLE = [  # (prediction row, positive mask row, k, expected NDCG)  tests/test_ndcg.py:10-21
    ([5, 4, 3, 2, 1], [1, 0, 0, 0, 0], 1, 1.0), ([4, 5, 3, 2, 1], [1, 0, 0, 0, 0], 1, 0.0),
    ([5, 4, 3, 2, 1], [1, 0, 0, 0, 0], 3, 1.0), ([4, 5, 3, 2, 1], [1, 0, 0, 0, 0], 3, 0.6309),
    ([3, 4, 5, 2, 1], [1, 0, 0, 0, 0], 3, 0.5), ([5, 4, 3, 2, 1], [1, 0, 0, 0, 0], 5, 1.0),
    ([4, 5, 3, 2, 1], [1, 0, 0, 0, 0], 5, 0.6309), ([3, 4, 5, 2, 1], [1, 0, 0, 0, 0], 5, 0.5),
    ([2, 3, 4, 5, 1], [1, 0, 0, 0, 0], 5, 0.4306), ([1, 2, 3, 4, 5], [1, 0, 0, 0, 0], 5, 0.3868),
]
MULTI = [  # tests/test_ndcg.py:24-35
    ([0, 0, 0, 4, 5], [0, 0, 0, 1, 1], 2, 1.0), ([0, 0, 4, 5, 0], [0, 0, 0, 1, 1], 2, 1. / (1. + 0.6309)),
    ([0, 4, 5, 0, 0], [0, 0, 0, 1, 1], 2, 0.0), ([0, 0, 0, 4, 5], [0, 0, 0, 1, 0], 2, 0.6309),
    ([0, 3, 4, 0, 5], [0, 0, 1, 1, 1], 2, 1.0),
    ([0, 3, 4, 0, 5], [0, 0, 1, 1, 1], 3, (1. + 0.6309) / (1. + 0.6309 + 0.5)),
    ([0, 3, 4, 0, 5], [1, 0, 0, 0, 1], 2, 1. / (1. + 0.6309)),
]


@pytest.mark.parametrize("pred,mask,k,want", SINGLE)
def test_ndcg_single_item(asme, pred, mask, k, want):
    p, m = np.array([pred], np.float32), np.array([mask])
    assert abs(O.ndcg_at_k(O.target_ranks(p, m.argmax(1)), k)[0] - want) < EPS
    assert abs(O.ndcg_multi(p, m, k)[0] - want) < EPS
    metric = asme.metrics.NormalizedDiscountedCumulativeGainMetric(k=k)
    metric.update(torch.tensor(p), torch.tensor(m))  # host tensors -> the host (top-k) path
    assert abs(float(metric.compute()) - want) < EPS


@pytest.mark.parametrize("pred,mask,k,want", MULTI)
def test_ndcg_multi_item(asme, pred, mask, k, want):
    p, m = np.array([pred], np.float32), np.array([mask])
    # rows with zero-score ties: the expected values are tie-order independent for these samples
    assert abs(O.ndcg_multi(p, m, k)[0] - want) < EPS
    metric = asme.metrics.NormalizedDiscountedCumulativeGainMetric(k=k)
    metric.update(torch.tensor(p), torch.tensor(m))
    assert abs(float(metric.compute()) - want) < EPS


def test_recall_and_mrr_host_path(asme):
    p = torch.tensor([[3., 4., 5., 2., 1.], [5., 4., 3., 2., 1.]])
    m = torch.tensor([[1, 0, 0, 0, 0], [0, 1, 0, 0, 0]])
    r = asme.metrics.RecallMetric(k=3)
    r.update(p, m)
    assert abs(float(r.compute()) - 1.0) < EPS
    mrr = asme.metrics.MRRMetric(k=3)
    mrr.update(p, m)
    assert abs(float(mrr.compute()) - (1 / 3 + 1 / 2) / 2) < EPS


# ---- input producers: the reference's own processor KATs (tests/test_cloze_mask.py,
# tests/test_pos_neg.py, seed_everything(42) -> torch's CPU generator; the example vocabulary has 13 ids,
# specials PAD=0 MASK=1 UNK=2), reproduced by the oracle's restatement of the processors
def test_oracle_cloze_mask_reference_kats():
    import torch
    from oracle import asme_oracle as O
    torch.manual_seed(42)
    seq, tgt = O.cloze_mask([5, 8, 9, 7, 3, 4], 1.0, 1.0, 13)
    assert seq == [5, 8, 9, 7, 3, 1] and tgt == [0] * 5 + [4]
    torch.manual_seed(42)
    seq, tgt = O.cloze_mask([5, 8, 9, 7, 3, 4, 12, 10, 11, 3], 0.5, 0.1, 13)
    assert seq == [5, 1, 9, 1, 3, 1, 12, 10, 1, 3]
    assert tgt == [0, 8, 0, 7, 0, 4, 0, 0, 11, 0]


def test_oracle_pos_neg_reference_kat():
    import torch
    from oracle import asme_oracle as O
    torch.manual_seed(42)
    x, pos, neg = O.pos_neg([5, 8, 9, 7, 3, 4], 13, [0, 1, 2])
    assert x == [5, 8, 9, 7, 3] and pos == [8, 9, 7, 3, 4] and neg == [6, 6, 6, 6, 11]


def test_oracle_cloze_draws_replay():
    """cloze_draws lays the generator's draws out per (session, position): applying the processor's decision
    rule to that layout reproduces cloze_mask run on the generator itself (what asme_cloze_mask's replay mode
    relies on)"""
    import numpy as np
    import torch
    from oracle import asme_oracle as O
    g = np.random.default_rng(0)
    sessions = [[int(v) for v in g.integers(3, 50, size=int(n))] for n in g.integers(1, 30, size=60)]
    torch.manual_seed(7)
    ref = [O.cloze_mask(s, 0.3, 0.1, 50) for s in sessions]
    torch.manual_seed(7)
    u, r = O.cloze_draws([len(s) for s in sessions], 30, 0.3, 0.1, 50)
    for b, s in enumerate(sessions):
        out, tgt = list(s), [0] * len(s)
        if float(u[b, 0]) <= 0.1:
            out[-1], tgt[-1] = 1, s[-1]
        else:
            for i in range(len(s)):
                p = float(u[b, 1 + i])
                if p < 0.3:
                    q = p / 0.3
                    out[i] = 1 if q < 0.8 else (int(r[b, i]) if q < 0.9 else s[i])
                    tgt[i] = s[i]
        assert (out, tgt) == ref[b], b


def test_oracle_last_item_mask_reference_example():
    """the processor's own docstring example (last_item_mask.py:13-19): [1, 5, 7, 8] -> [1, 5, 7, 8, 101]"""
    assert O.last_item_mask([1, 5, 7, 8], mask_id=101) == [1, 5, 7, 8, 101]
    assert O.collate_pad(O.last_item_mask([1, 5, 7, 8], mask_id=101), 3, pad=0) == [7, 8, 101]
