"""The SASRec step's table ids deduplicated a step ahead on a side stream (module.prefetch -> ops.TableIdsAhead:
dedup + occurrence CSR over the module's spare slot map, the training stream waiting for them) must train exactly
like the inline dedup -- same kernels on the same ids, so every loss, parameter and Adam moment is bit-identical --
including a prefetch of a batch the next step does not take (discarded, its map entries reset) and prefetches of
Zipf-like ids whose hot rows take the CSR's long-list path.  Reference path: the sampler + module of
/root/reference/src/asme/data/datasets/processors/pos_neg_sampler.py:41-106 and
core/modules/next_item_prediction_training_module.py (the SASRec step), bench.py's SASRec leg."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(asme, dev, V, L, d, hot):
    torch.manual_seed(0)
    n_sess = 96
    g = torch.Generator(device=dev).manual_seed(11)
    if hot:  # a few very frequent ids (hot keys: occurrence lists beyond 256)
        flat = torch.where(torch.rand(n_sess * (L + 1), device=dev, generator=g) < 0.5,
                           torch.randint(3, 8, (n_sess * (L + 1),), device=dev, generator=g),
                           torch.randint(3, V, (n_sess * (L + 1),), device=dev, generator=g))
    else:
        flat = torch.randint(3, V, (n_sess * (L + 1),), device=dev, generator=g)
    store = asme.batches.SessionStore(flat, torch.arange(n_sess + 1, device=dev) * (L + 1))
    tok = asme.tokenization.Tokenizer(V - 3)
    sampler = asme.batches.PositiveNegativeSamplerProcessor(tok)
    return store, tok, sampler


def _train(asme, dev, mode, steps=6, V=5003, B=32, L=50, d=64, hot=False):
    store, tok, sampler = _setup(asme, dev, V, L, d, hot)
    torch.manual_seed(1)
    with torch.device(dev):
        model = asme.SASRecModel(transformer_hidden_size=d, num_transformer_heads=2, num_transformer_layers=2,
                                 item_vocab_size=V, max_seq_length=L, transformer_dropout=0.1)
    module = asme.SequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=None)
    module.train()
    opt = module.configure_optimizers()
    side = torch.cuda.Stream(dev)

    def get_batch(i):
        idx = torch.arange(B, device=dev) + (i * B) % (96 - B)
        b = sampler.process_batch(store, idx, L, seed=500 + i)
        return {k: b[k] for k in ("item", "positive_samples", "negative_samples")}

    losses, ahead = [], {}
    torch.manual_seed(2)  # the dropout seeds: drawn in the same order by both forms
    for j in range(steps):
        b = ahead.pop(j, None)
        if b is None:
            b = get_batch(j)
        losses.append(asme.modules.train_step(module, opt, None, b, j).detach())
        if mode != "inline" and j + 1 < steps:
            with torch.cuda.stream(side):
                nb = get_batch(j + 1)
                if mode == "mismatch" and j % 2 == 0:
                    module.prefetch(get_batch(j + 1))  # ids the next step will not take: discarded there
                else:
                    module.prefetch(nb)
            ahead[j + 1] = nb
    torch.cuda.synchronize()
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}  # (flushes the lazily updated rows)
    st = opt.state[model.item_table()]
    return torch.stack(losses).cpu(), sd, (st["exp_avg"].cpu(), st["exp_avg_sq"].cpu()), module.ids_ahead_hits


@pytest.mark.parametrize("hot", [False, True])
def test_ids_ahead_training_is_bit_identical(asme, dev, hot):
    ref = _train(asme, dev, "inline", hot=hot)
    got = _train(asme, dev, "ahead", hot=hot)
    assert ref[3] == 0 and got[3] == 5  # every step after the first took its dedup from the side stream
    assert torch.equal(got[0], ref[0])
    for k in ref[1]:
        assert torch.equal(got[1][k], ref[1][k]), k
    assert torch.equal(got[2][0], ref[2][0]) and torch.equal(got[2][1], ref[2][1])


def test_ids_ahead_mismatched_prefetch_is_discarded(asme, dev):
    ref = _train(asme, dev, "inline")
    got = _train(asme, dev, "mismatch")
    assert got[3] == 2  # steps 2 and 4 took theirs; 1, 3 and 5 got a batch other than the prefetched one
    assert torch.equal(got[0], ref[0])
    for k in ref[1]:
        assert torch.equal(got[1][k], ref[1][k]), k


def test_ids_ahead_plan_equals_inline_plan(asme, dev):
    """the ahead half alone: unique ids, inverse and count equal the inline dedup's, the CSR is built on the
    ahead stream, and the spare map is clean again after the plan's release"""
    V, n = 7001, 3000
    gen = torch.Generator(device=dev).manual_seed(3)
    ids = [torch.randint(0, V, (n,), device=dev, generator=gen) for _ in range(3)]
    m_in = asme.ops.new_slot_map(V, dev)
    m_ah = asme.ops.new_slot_map(V, dev)
    inline = asme.ops.SparseTablePlan(None, ids, m_in, vocab=V, dim=32)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        ah = asme.ops.TableIdsAhead(V, 32, ids, m_ah)
    plan = asme.ops.SparseTablePlan(None, ids, m_ah, vocab=V, dim=32, ahead=ah)
    assert plan._csr is not None
    assert torch.equal(plan.count, inline.count)
    c = int(inline.count.item())
    assert torch.equal(plan.unique[:c], inline.unique[:c])
    for x in ids:
        assert torch.equal(plan.inverse_of(x), inline.inverse_of(x))
    with pytest.raises(ValueError):
        asme.ops.SparseTablePlan(None, ids[:2], m_ah, vocab=V, dim=32, ahead=ah)
    plan.release()
    inline.release()
    torch.cuda.synchronize()
    assert bool((m_ah == -1).all()) and bool((m_in == -1).all())
