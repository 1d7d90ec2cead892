"""MaskedTrainingModule.prefetch: the next step's masked rows selected ahead on a side stream give the very same
training step as selecting them inside training_step (bit-identical loss and gradients), and a batch other than the
prefetched one falls back to the in-step selection."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _module(asme, dev, seed):
    torch.manual_seed(seed)
    V = 503
    with torch.device(dev):
        model = asme.BERT4RecModel(transformer_hidden_size=32, num_transformer_heads=2, num_transformer_layers=1,
                                   item_vocab_size=V, max_seq_length=20, transformer_dropout=0.0)
    tok = asme.tokenization.Tokenizer(V - 3)
    return asme.MaskedTrainingModule(model=model, item_tokenizer=tok, metrics=None), tok, V


def test_masked_rows_prefetch_matches_inline(asme, dev):
    (m1, tok, V), (m2, _, _) = _module(asme, dev, 3), _module(asme, dev, 3)
    g = torch.Generator(device=dev).manual_seed(7)
    items = torch.randint(3, V, (16, 20), device=dev, generator=g)
    lengths = torch.randint(2, 21, (16,), device=dev, generator=g)
    items = torch.where(torch.arange(20, device=dev) < lengths[:, None], items, 0)
    batch = asme.batches.ClozeMaskProcessor(tok, 0.2, 0.1).process_batch(items, lengths, seed=11)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        m2.prefetch(batch)
    torch.cuda.current_stream().wait_stream(side)
    l1 = m1.training_step(batch, 0)["loss"]
    l2 = m2.training_step(batch, 0)["loss"]
    assert m2._rows_ahead is None  # consumed
    l1.backward()
    l2.backward()
    assert torch.equal(l1, l2)
    for p1, p2 in zip(m1.parameters(), m2.parameters()):
        assert (p1.grad is None) == (p2.grad is None)
        if p1.grad is not None:
            assert torch.equal(p1.grad, p2.grad)
    # a prefetch of another batch is not used (the step selects its own rows)
    other = {k: v.clone() for k, v in batch.items()}
    m2.prefetch(other)
    l3 = m2.training_step(batch, 1)["loss"]
    assert torch.equal(l3, m1.training_step(batch, 1)["loss"])
