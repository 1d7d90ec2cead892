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
