"""FusedAdam state handling with the lazily-updated item table (ops.LazyTableState):
resume at a large step, optimizer state_dict round trips, and dataloader ids of other dtypes."""
import copy

import pytest
import torch

from helpers import build_model, load, state_dict

pytestmark = pytest.mark.gpu


def _sasrec(asme, dev, table_grad):
    z = load("sasrec_neg")
    model = build_model(asme, "sasrec_neg", z)
    model.load_state_dict(state_dict(z))
    model.to(dev)
    tok = asme.tokenization.Tokenizer(int(z["cfg"][5]) - 3)
    module = asme.SequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=None,
                                                           table_grad=table_grad)
    batch = {k: torch.from_numpy(z[s]).to(dev) for k, s in
             (("item", "seq"), ("positive_samples", "pos"), ("negative_samples", "neg"))}
    return model, module, batch


def _params(model):
    return {k: v.detach().clone() for k, v in model.state_dict().items()}  # state_dict() flushes the table


def test_default_table_grad_is_sparse_for_gather_only_tables(asme, dev):
    _, module, _ = _sasrec(asme, dev, None)
    assert module.table_grad == "sparse"


def test_lazy_table_resumed_at_large_step(asme, dev):
    """a run resumed at step 5000 (beyond the first history capacity) takes the same sparse/lazy step as the
    eager row update (the history buffer must grow to step + 1 at once)"""
    results = []
    for lazy in (True, False):
        model, module, batch = _sasrec(asme, dev, "sparse")
        opt = asme.FusedAdam(module.parameters(), lr=1e-3, betas=(0.99, 0.998), weight_decay=1e-3, lazy_table=lazy)
        for p in module.parameters():  # pretend 5000 steps were taken: moments and step counts of a checkpoint
            st = opt._state(p)
            st["step"] = 5000
            st["exp_avg"].fill_(1e-4)
            st["exp_avg_sq"].fill_(1e-6)
        for i in range(2):
            asme.modules.train_step(module, opt, None, batch, i)
        opt.flush()
        table = model.item_table()
        assert opt.state[table]["step"] == 5002
        results.append(_params(model))
    for k in results[0]:
        assert torch.equal(results[0][k], results[1][k]), k


def test_optimizer_state_dict_round_trip(asme, dev):
    """save -> load -> step reproduces the uninterrupted run bit for bit (the lazy table state is rebuilt
    from the loaded moments; state_dict() flushes the deferred rows first)"""
    model, module, batch = _sasrec(asme, dev, "sparse")
    opt = module.configure_optimizers()
    for i in range(3):
        asme.modules.train_step(module, opt, None, batch, i)
    saved_opt = copy.deepcopy(opt.state_dict())
    saved_model = _params(model)
    for i in range(2):
        asme.modules.train_step(module, opt, None, batch, 3 + i)
    straight = _params(model)
    # rewind the same model and optimizer
    model.load_state_dict(saved_model)
    opt.load_state_dict(saved_opt)
    assert all(getattr(p, "_asme_table_grad", None) is None or p._asme_table_grad.lazy is None
               for p in module.parameters())
    for i in range(2):
        asme.modules.train_step(module, opt, None, batch, 3 + i)
    resumed = _params(model)
    for k in straight:
        assert torch.equal(straight[k], resumed[k]), k


def test_state_dict_moments_are_current(asme, dev):
    """optimizer.state_dict() without a model.state_dict() first must not return stale table moments"""
    res = {}
    for mode in ("sparse", "dense"):
        model, module, batch = _sasrec(asme, dev, mode)
        opt = module.configure_optimizers()
        for i in range(3):
            asme.modules.train_step(module, opt, None, batch, i)
        sd = opt.state_dict()
        idx = [i for i, p in enumerate(module.parameters()) if p is model.item_table()][0]
        res[mode] = sd["state"][idx]["exp_avg"].clone()
    assert (res["sparse"] - res["dense"]).abs().max().item() <= 1e-5 * res["dense"].abs().max().item()


def test_int32_batch_ids_with_sparse_table(asme, dev):
    """int32 dataloader ids: the plan registers the normalised tensors the model reads"""
    out = []
    for dtype in (torch.int64, torch.int32):
        model, module, batch = _sasrec(asme, dev, "sparse")
        batch = {k: v.to(dtype) for k, v in batch.items()}
        opt = module.configure_optimizers()
        for i in range(2):
            asme.modules.train_step(module, opt, None, batch, i)
        out.append(_params(model))
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k


def test_staged_rows_match_in_place_catch_up(asme, dev, monkeypatch):
    """lazy table Adam with the step's rows staged in slot order (asme_lazy_adam_stage / _apply_staged, every
    reader gathering the staged rows) == catching them up in place in the table, bit for bit -- across a
    flush between forward and step (state_dict), a re-step without a new backward and a resumed step count; the
    staged step both fused with the gradient reduction (asme_table_grad_reduce_apply) and separate"""
    out = []
    for staged, fused in ((True, True), (True, False), (False, True)):
        monkeypatch.setattr(asme.ops, "STAGE_ROWS", staged)
        model, module, batch = _sasrec(asme, dev, "sparse")
        opt = module.configure_optimizers()
        opt.fused_apply = fused  # FusedAdam(fused_apply=...)
        seen = []
        for i in range(4):
            module.train()
            loss = module.training_step(batch, i)["loss"]
            table = model.item_table()
            seen.append(table._asme_table_grad.plan.staged is not None)
            if i == 2:
                model.state_dict()  # flush while the step's rows are staged
            loss.backward()
            opt.step()
            if i == 1:
                opt.step()  # re-step: the kept gradient again, rows caught up from the table
            opt.zero_grad()
        assert seen == [False, staged, staged, staged]
        out.append(_params(model))
        out.append({k: v.clone() for k, v in opt.state[model.item_table()].items() if torch.is_tensor(v)})
    for a, b in ((out[0], out[4]), (out[1], out[5]), (out[2], out[4]), (out[3], out[5])):
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_skipped_optimizer_step_drops_the_table_gradient(asme, dev):
    """a backward whose optimizer step is skipped (a GradScaler inf/NaN skip, a trainer skipping the step) drops the
    row-sparse table gradient, as zero_grad drops a dense one: the next step equals a run without the skipped
    backward.  Without that zero_grad (gradient accumulation: a second training_step + backward before the step)
    the next training_step raises instead of dropping or merging the first table gradient."""
    out = []
    for skip in (False, True):
        model, module, batch = _sasrec(asme, dev, "sparse")
        opt = module.configure_optimizers()
        if skip:
            module.training_step(batch, 0)["loss"].backward()   # no optimizer step follows
            opt.zero_grad()
        asme.modules.train_step(module, opt, None, batch, 0)
        out.append(_params(model))
    for k in out[0]:
        assert torch.equal(out[0][k], out[1][k]), k
    model, module, batch = _sasrec(asme, dev, "sparse")
    opt = module.configure_optimizers()
    module.training_step(batch, 0)["loss"].backward()
    with pytest.raises(RuntimeError, match="gradient accumulation"):
        module.training_step(batch, 1)
    # zero_grad between training_step and backward (Lightning's closure order) keeps the step's plan
    model, module, batch = _sasrec(asme, dev, "sparse")
    opt = module.configure_optimizers()
    loss = module.training_step(batch, 0)["loss"]
    opt.zero_grad()
    asme.modules.backward(loss)
    opt.step()
    opt.zero_grad()
    assert _params(model).keys() == out[0].keys()
    for k in out[0]:
        assert torch.equal(_params(model)[k], out[0][k]), k
