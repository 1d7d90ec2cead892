"""GPU batch producers (csrc/batch.hip, asme_amd.batches) against the oracle's restatement of the reference's
processors (oracle/asme_oracle.py: cloze_mask, pos_neg, last_item_mask, collate_pad), which itself reproduces the reference's
own known-answer tests (tests/test_reference_kats.py).

Cloze masking replays the reference's torch CPU generator stream (oracle.cloze_draws) and must match the
processor bit-exactly, KAT sessions included.  The negative sampler draws from its own Philox stream (the
reference's torch.multinomial stream cannot be replayed on the GPU): x / pos / padding are checked bit-exactly,
negatives by the sampler's contract (never special, never in the session, uniform over the admissible ids) and
by determinism per seed."""
import numpy as np
import pytest
import torch

from oracle import asme_oracle as O

pytestmark = pytest.mark.gpu


def _tok(asme, V):
    return asme.tokenization.Tokenizer(V - 3)


def _collated(sessions, L, pad=0):
    items = torch.tensor([O.collate_pad(s, L, pad) for s in sessions], dtype=torch.int64)
    lengths = torch.tensor([min(len(s), L) for s in sessions], dtype=torch.int64)
    return items, lengths


@pytest.mark.parametrize("seed,mask_prob,last_prob", [(7, 0.3, 0.1), (11, 0.2, 0.1), (3, 0.5, 0.0), (5, 1.0, 0.5)])
def test_cloze_replay_matches_reference_processor(asme, dev, seed, mask_prob, last_prob):
    V, L = 60, 24
    g = np.random.default_rng(seed)
    sessions = [[int(v) for v in g.integers(3, V, size=int(n))] for n in g.integers(1, L + 1, size=300)]
    torch.manual_seed(seed)
    ref = [O.cloze_mask(s, mask_prob, last_prob, V) for s in sessions]
    torch.manual_seed(seed)
    u, r = O.cloze_draws([len(s) for s in sessions], L, mask_prob, last_prob, V)
    proc = asme.batches.ClozeMaskProcessor({"tokenizers.item": _tok(asme, V)}, mask_prob, last_prob)
    items, lengths = _collated(sessions, L)
    out = proc.process_batch(items.to(dev), lengths.to(dev), draws=(torch.from_numpy(u), torch.from_numpy(r)))
    want_x = torch.tensor([O.collate_pad(x, L) for x, _ in ref])
    want_t = torch.tensor([O.collate_pad(t, L) for _, t in ref])
    assert torch.equal(out["item"].cpu(), want_x)
    assert torch.equal(out["item.target"].cpu(), want_t)


def test_cloze_reference_kat_sessions(asme, dev):
    """the reference's tests/test_cloze_mask.py sessions and expected outputs (seed 42, 13-id vocabulary)"""
    for sess, p, pl, want_x, want_t in (
            ([5, 8, 9, 7, 3, 4], 1.0, 1.0, [5, 8, 9, 7, 3, 1], [0] * 5 + [4]),
            ([5, 8, 9, 7, 3, 4, 12, 10, 11, 3], 0.5, 0.1, [5, 1, 9, 1, 3, 1, 12, 10, 1, 3],
             [0, 8, 0, 7, 0, 4, 0, 0, 11, 0])):
        L = len(sess)
        torch.manual_seed(42)
        u, r = O.cloze_draws([L], L, p, pl, 13)
        proc = asme.batches.ClozeMaskProcessor({"tokenizers.item": _tok(asme, 13)}, p, pl)
        out = proc.process_batch(torch.tensor([sess], device=dev), torch.tensor([L], device=dev),
                                 draws=(torch.from_numpy(u), torch.from_numpy(r)))
        assert out["item"].cpu().tolist() == [want_x]
        assert out["item.target"].cpu().tolist() == [want_t]


def test_cloze_philox_statistics_and_determinism(asme, dev):
    V, L, B = 27003, 200, 4096
    p, pl = 0.2, 0.1
    items = torch.randint(3, V, (B, L), device=dev)
    lengths = torch.full((B,), L, device=dev)
    proc = asme.batches.ClozeMaskProcessor({"tokenizers.item": _tok(asme, V)}, p, pl)
    a = proc.process_batch(items, lengths, seed=1234)
    b = proc.process_batch(items, lengths, seed=1234)
    c = proc.process_batch(items, lengths, seed=4321)
    assert torch.equal(a["item"], b["item"]) and torch.equal(a["item.target"], b["item.target"])
    assert not torch.equal(a["item"], c["item"])
    x, t = a["item"], a["item.target"]
    masked = t != 0
    last_only = masked[:, :-1].sum(1).eq(0) & masked[:, -1] & x[:, -1].eq(1)
    assert abs(last_only.float().mean().item() - pl) < 0.02
    rest = ~last_only
    frac = masked[rest].float().mean().item()
    assert abs(frac - p) < 0.01
    m = masked & rest.unsqueeze(1)
    n_mask = (x[m] == 1).float().mean().item()
    n_keep = (x[m] == items[m]).float().mean().item()
    assert abs(n_mask - 0.8) < 0.01 and abs(n_keep - 0.1 - 1.0 / V) < 0.01
    rnd = x[m][(x[m] != 1) & (x[m] != items[m])]
    assert int(rnd.min()) >= 0 and int(rnd.max()) < V - 1
    assert torch.equal(t[masked], items[masked])


def test_padded_session_batch_matches_collate(asme, dev):
    g = np.random.default_rng(1)
    sessions = [[int(v) for v in g.integers(3, 500, size=int(n))] for n in g.integers(1, 90, size=200)]
    store = asme.batches.SessionStore.from_lists(sessions, dev)
    idx = torch.tensor(g.permutation(len(sessions))[:128], dtype=torch.int64)
    out, lengths = asme.batches.padded_session_batch(store, idx.to(dev), 50)
    want = torch.tensor([O.collate_pad(sessions[i], 50) for i in idx.tolist()])
    assert torch.equal(out.cpu(), want)
    assert lengths.cpu().tolist() == [min(len(sessions[i]), 50) for i in idx.tolist()]


@pytest.mark.parametrize("L_in,L_out", [(50, 50), (49, 50), (64, 20)])
def test_last_item_mask_matches_processor_then_collate(asme, dev, L_in, L_out):
    """LastItemMaskProcessor (MASK appended to the session) then the collate (left truncation to L_out, right
    padding), against the oracle restatement applied to the full sessions; lengths 0..L_out+ covered"""
    g = np.random.default_rng(L_in + L_out)
    sessions = [[int(v) for v in g.integers(3, 500, size=int(n))] for n in list(range(0, 80)) + [L_out - 1, L_out]]
    V = 600
    tok = _tok(asme, V)
    items, lengths = _collated(sessions, L_in, tok.pad_token_id)
    proc = asme.batches.LastItemMaskProcessor({"item": tok})
    out, out_len = proc.process_batch(items.to(dev), lengths.to(dev), L_out)
    want = [O.collate_pad(O.last_item_mask(s, tok.mask_token_id), L_out, tok.pad_token_id) for s in sessions]
    assert out.cpu().tolist() == want
    assert out_len.cpu().tolist() == [min(len(s) + 1, L_out) for s in sessions]


def test_posneg_sampler_contract(asme, dev):
    V, L = 1000, 50
    g = np.random.default_rng(2)
    sessions = [[int(v) for v in g.choice(np.arange(3, V), size=int(n), replace=False)]
                for n in g.integers(2, 150, size=300)]
    store = asme.batches.SessionStore.from_lists(sessions, dev)
    proc = asme.batches.PositiveNegativeSamplerProcessor({"tokenizers.item": _tok(asme, V)})
    idx = torch.arange(len(sessions), device=dev)
    a = proc.process_batch(store, idx, L, seed=99)
    b = proc.process_batch(store, idx, L, seed=99)
    proc.check_errors()
    assert all(torch.equal(a[k], b[k]) for k in a)
    for i, s in enumerate(sessions):
        x, pos, _ = s[:-1], s[1:], None
        assert a["item"][i].tolist() == O.collate_pad(x, L)
        assert a["positive_samples"][i].tolist() == O.collate_pad(pos, L)
        n = min(len(s) - 1, L)
        negs = a["negative_samples"][i, :n].tolist()
        assert all(v >= 3 and v < V and v not in set(s) for v in negs), i
        assert a["negative_samples"][i, n:].eq(0).all()
        assert int(a["length"][i]) == n


def test_posneg_sampler_uniform_over_admissible(asme, dev):
    """tiny vocabulary: the negatives of one session are uniform over the ids neither special nor in it"""
    V, L = 20, 40
    sess = [3, 7, 7, 11, 15]
    sessions = [sess] * 2000
    store = asme.batches.SessionStore.from_lists(sessions, dev)
    proc = asme.batches.PositiveNegativeSamplerProcessor({"tokenizers.item": _tok(asme, V)})
    out = proc.process_batch(store, torch.arange(len(sessions), device=dev), L, seed=5)
    negs = out["negative_samples"][:, :4].reshape(-1).cpu()
    allowed = [v for v in range(3, V) if v not in sess]
    counts = torch.bincount(negs, minlength=V)
    assert int(counts[[v for v in range(V) if v not in allowed]].sum()) == 0
    expect = negs.numel() / len(allowed)
    chi2 = float(((counts[allowed].double() - expect) ** 2 / expect).sum())
    assert chi2 < 45.0  # 13 dof, p ~ 1e-5


def test_posneg_sampler_errors(asme, dev):
    V = 8  # specials 0, 1, 2; items 3..7
    tok = _tok(asme, V)
    proc = asme.batches.PositiveNegativeSamplerProcessor({"tokenizers.item": tok})
    store = asme.batches.SessionStore.from_lists([[3, 4], [5]], dev)
    proc.process_batch(store, torch.tensor([0, 1], device=dev), 4, seed=1)
    with pytest.raises(AssertionError):
        proc.check_errors()
    store = asme.batches.SessionStore.from_lists([[3, 4, 5, 6, 7]], dev)
    proc.process_batch(store, torch.tensor([0], device=dev), 4, seed=1)
    with pytest.raises(RuntimeError):
        proc.check_errors()
