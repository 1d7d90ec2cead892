"""Generate golden fixtures by running the READ-ONLY reference (ASME) on CPU.

Build-container only (needs /root/reference); the GPU box and the product never run
this.  Every fixture is data: a seeded synthetic batch, the reference model's
state_dict, and the reference's outputs / losses / gradients / optimizer results,
written as small .npz files under tests/golden/.  Which reference code produced each
array is noted next to it (paths relative to /root/reference/src/asme).

    python tests/golden/make_golden.py            # all fixtures
    python tests/golden/make_golden.py ml1m       # only the ml-1m-shaped NDCG anchor
    python tests/golden/make_golden.py ddp        # the DDP (multi-rank) fixtures, W = 2 and 8
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _ref_stubs as S  # noqa: E402

S.install()
import torch  # noqa: E402

torch.set_num_threads(1)
PAD, MASK = 0, 1


def _sd(model):
    # keep every key, shared modules included (checkpoint-compatible key names)
    return {f"sd/{k}": v.detach().cpu().numpy().copy() for k, v in model.state_dict(keep_vars=False).items()}


def _grads(model):
    return {f"grad/{n}": (p.grad.detach().numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32))
            for n, p in model.named_parameters()}


def _params(model, prefix):
    return {f"{prefix}/{n}": p.detach().numpy().copy() for n, p in model.named_parameters()}


def _ragged_batch(g, B, L, V, lengths):
    seq = torch.zeros(B, L, dtype=torch.long)
    for b, n in enumerate(lengths):
        seq[b, :n] = torch.randint(3, V, (n,), generator=g)
    return seq


def _hook_outputs(model):
    out = {}

    def emb_hook(mod, inp, res):
        out["emb_out"] = res.embedded_sequence.detach().clone()

    def rep_hook(mod, inp, res):
        out["enc_out"] = res.encoded_sequence.detach().clone()

    model._sequence_embedding_layer.register_forward_hook(emb_hook)
    model._sequence_representation_layer.register_forward_hook(rep_hook)
    return out


# ----------------------------------------------------------------------------------
def gen_sasrec_neg(B=4, L=12, d=32, h=2, N=2, NI=57, lengths=(12, 9, 5, 1), suffix=""):
    """sasrec-neg: SequenceNextItemPredictionTrainingModule + SASRecModel(mode=neg_sampling)
    core/modules/sequence_next_item_prediction_training_module.py:73-115,156-185
    core/models/sasrec/sasrec_model.py:29-108, core/models/sasrec/components.py:21-61
    core/losses/sasrec/sas_rec_losses.py:35-75"""
    tok = S.make_tokenizer(NI)
    S.set_context({"item": tok})
    from asme.core.models.sasrec.sasrec_model import SASRecModel
    from asme.core.modules.sequence_next_item_prediction_training_module import \
        SequenceNextItemPredictionTrainingModule
    V = len(tok)
    torch.manual_seed(0)
    model = SASRecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                        max_seq_length=L, transformer_dropout=0.0)
    module = SequenceNextItemPredictionTrainingModule(model=model, metrics=None)
    sd = _sd(model)
    g = torch.Generator().manual_seed(1)
    lengths = list(lengths)
    full = _ragged_batch(g, B, L + 1, V, [n + 1 for n in lengths])
    seq = full[:, :L].clone()
    pos = full[:, 1:].clone()
    for b, n in enumerate(lengths):
        seq[b, n:] = PAD
        pos[b, n:] = PAD
    neg = torch.randint(3, V, (B, L), generator=g)
    neg[seq == PAD] = PAD
    hooks = _hook_outputs(model)
    batch = {"item": seq, "positive_samples": pos, "negative_samples": neg}
    res = module.training_step(batch, 0)
    loss = res["loss"]
    # pos/neg logits from the model directly (same forward as training_step)
    from asme.core.models.common.layers.data.sequence import InputSequence
    with torch.no_grad():
        pl, nl = model(InputSequence(seq, seq.ne(PAD), {"positive_samples": pos, "negative_samples": neg}))
    loss.backward()
    grads = _grads(model)
    opt = module.configure_optimizers()
    opt.step()
    after = _params(model, "adam1")
    # eval (full catalogue, predict_step): uses the updated params -> reload original first
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    with torch.no_grad():
        pred = module.predict_step({"item": seq}, 0)
    out = dict(sd)
    out.update(grads)
    out.update(after)
    out.update(dict(seq=seq.numpy(), pos=pos.numpy(), neg=neg.numpy(), pos_logits=pl.numpy(), neg_logits=nl.numpy(),
                    loss=loss.detach().numpy(), emb_out=hooks["emb_out"].numpy(), enc_out=hooks["enc_out"].numpy(),
                    eval_logits=pred.numpy(),
                    cfg=np.array([B, L, d, h, N, V]), lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32),
                    weight_decay=np.float32(1e-3)))
    np.savez_compressed(os.path.join(HERE, f"sasrec_neg{suffix}.npz"), **out)
    print("sasrec_neg" + suffix, float(loss))


def gen_sasrec_cross(B=4, L=10, d=32, h=2, N=2, NI=45, lengths=(10, 7, 3, 2), suffix=""):
    """sasrec-cross: NextItemPredictionTrainingModule + SASRecModel(mode=full)
    core/modules/next_item_prediction_training_module.py:141-256
    core/losses/sasrec/sas_rec_losses.py:9-32, core/models/common/layers/layers.py:92-109"""
    tok = S.make_tokenizer(NI)
    S.set_context({"item": tok})
    from asme.core.models.sasrec.sasrec_model import SASRecModel
    from asme.core.modules.next_item_prediction_training_module import NextItemPredictionTrainingModule
    from asme.core.losses.sasrec.sas_rec_losses import SASRecFullSequenceCrossEntropyLoss
    V = len(tok)
    torch.manual_seed(2)
    model = SASRecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                        max_seq_length=L, transformer_dropout=0.0, mode="full")
    module = NextItemPredictionTrainingModule(model=model, metrics=None,
                                              loss_function=SASRecFullSequenceCrossEntropyLoss)
    sd = _sd(model)
    g = torch.Generator().manual_seed(3)
    lengths = list(lengths)
    full = _ragged_batch(g, B, L + 1, V, [n + 1 for n in lengths])
    seq = full[:, :L].clone()
    tgt = full[:, 1:].clone()
    for b, n in enumerate(lengths):
        seq[b, n:] = PAD
        tgt[b, n:] = PAD
    hooks = _hook_outputs(model)
    res = module.training_step({"item": seq, "item.target": tgt}, 0)
    loss = res["loss"]
    loss.backward()
    grads = _grads(model)
    opt = module.configure_optimizers()
    opt.step()
    after = _params(model, "adam1")
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    with torch.no_grad():
        logits = module({"item": seq}, 0)
        last = module.predict_step({"item": seq}, 0)
    out = dict(sd)
    out.update(grads)
    out.update(after)
    head = 16 if suffix else L  # the d = 128 fixture keeps the first 16 positions' logits
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), logits=logits[:, :head].numpy(), loss=loss.detach().numpy(),
                    emb_out=hooks["emb_out"].numpy(), enc_out=hooks["enc_out"].numpy(), eval_logits=last.numpy(),
                    logits_head=np.int64(head),
                    cfg=np.array([B, L, d, h, N, V]), lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32),
                    weight_decay=np.float32(0.0)))
    np.savez_compressed(os.path.join(HERE, f"sasrec_cross{suffix}.npz"), **out)
    print("sasrec_cross" + suffix, float(loss))


def _cloze_batch(g, B, L, V, lengths):
    seq = _ragged_batch(g, B, L, V, lengths)
    tgt = torch.zeros_like(seq)
    for b, n in enumerate(lengths):
        m = torch.rand(n, generator=g) < 0.3
        m[n - 1] = True
        tgt[b, :n][m] = seq[b, :n][m]
        seq[b, :n][m] = MASK
    return seq, tgt


def gen_bert4rec(kind: str, B=4, L=10, d=32, h=2, N=2, NI=47, lengths=(10, 8, 4, 2), suffix="", adam2=True):
    """bert4rec: MaskedTrainingModule + BERT4RecModel(project_layer_type=kind)
    core/modules/masked_training_module.py:20-189, core/models/bert4rec/bert4rec_model.py:24-68
    core/models/common/layers/layers.py:112-157, ffn_modifier.py:8-26"""
    tok = S.make_tokenizer(NI)
    S.set_context({"item": tok})
    from asme.core.models.bert4rec.bert4rec_model import BERT4RecModel
    from asme.core.modules.masked_training_module import MaskedTrainingModule
    V = len(tok)
    torch.manual_seed(4)
    model = BERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                          max_seq_length=L, transformer_dropout=0.0, project_layer_type=kind)
    module = MaskedTrainingModule(model=model, metrics=None, num_warmup_steps=10)
    sd = _sd(model)
    g = torch.Generator().manual_seed(5)
    lengths = list(lengths)
    seq, tgt = _cloze_batch(g, B, L, V, lengths)
    hooks = _hook_outputs(model)
    res = module.training_step({"item": seq, "item.target": tgt}, 0)
    loss = res["loss"]
    loss.backward()
    grads = _grads(model)
    opts, scheds = module.configure_optimizers()
    opt, sched = opts[0], scheds[0]["scheduler"]
    # two optimizer steps with the LambdaLR warmup (step 0 -> lr factor 0, step 1 -> 1/10)
    opt.step()
    sched.step()
    after1 = _params(model, "adam1")
    opt.step()
    sched.step()
    after2 = _params(model, "adam2") if adam2 else {}
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    # eval: one MASK at the last valid position (last_item_mask processor semantics)
    ev = seq.clone()
    ev[ev == MASK] = 7
    for b, n in enumerate(lengths):
        ev[b, n - 1] = MASK
    with torch.no_grad():
        logits = module({"item": seq}, 0)
        pred = module.predict_step({"item": ev}, 0)
    out = dict(sd)
    out.update(grads)
    out.update(after1)
    out.update(after2)
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), logits=logits[:, :16 if suffix else L].numpy(), loss=loss.detach().numpy(),
                    emb_out=hooks["emb_out"].numpy(), enc_out=hooks["enc_out"].numpy(),
                    eval_seq=ev.numpy(), eval_logits=pred.numpy(), num_warmup_steps=np.int64(10),
                    logits_head=np.int64(16 if suffix else L),
                    cfg=np.array([B, L, d, h, N, V]), lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32)))
    np.savez_compressed(os.path.join(HERE, f"bert4rec_{kind}{suffix}.npz"), **out)
    print("bert4rec", kind + suffix, float(loss))


def gen_kebert4rec(variant: str, B=4, L=10, d=32, h=2, N=2, NI=41, NG=7, NT=9, K=3, lengths=(10, 6, 5, 3),
                   suffix=""):
    """kebert4rec: MaskedTrainingModule + KeBERT4RecModel with attribute side-embeddings
    core/models/kebert4rec/kebert4rec_model.py:24-89, components.py:15-115, layers.py:7-27"""
    tok = S.make_tokenizer(NI)
    gtok = S.make_tokenizer(NG, "Genre")
    ttok = S.make_tokenizer(NT, "Tag")
    S.set_context({"item": tok, "genre": gtok, "tags": ttok})
    from asme.core.models.kebert4rec.kebert4rec_model import KeBERT4RecModel
    from asme.core.modules.masked_training_module import MaskedTrainingModule
    V = len(tok)
    if variant == "pre":
        pre = {"genre": {"embedding_type": "content_embedding"}, "tags": {"embedding_type": "linear_upscale"}}
        post = None
    else:
        pre = {"tags": {"embedding_type": "linear_upscale"}}
        post = {"genre": {"embedding_type": "content_embedding"}}
    torch.manual_seed(6)
    model = KeBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                            max_seq_length=L, transformer_dropout=0.0, prefusion_attributes=pre,
                            postfusion_attributes=post)
    module = MaskedTrainingModule(model=model, metrics=None, num_warmup_steps=0)
    sd = _sd(model)
    g = torch.Generator().manual_seed(7)
    lengths = list(lengths)
    seq, tgt = _cloze_batch(g, B, L, V, lengths)
    genre = torch.randint(3, len(gtok), (B, L), generator=g)
    tags = torch.randint(3, len(ttok), (B, L, K), generator=g)
    tags[:, :, 2][torch.rand(B, L, generator=g) < 0.5] = 0   # ragged multi-hot (0 = pad)
    genre[seq == PAD] = PAD
    tags[seq == PAD] = 0
    batch = {"item": seq, "item.target": tgt, "genre": genre, "tags": tags}
    hooks = _hook_outputs(model)
    res = module.training_step(batch, 0)
    loss = res["loss"]
    loss.backward()
    grads = _grads(model)
    opts = module.configure_optimizers()
    opts[0].step()
    after = _params(model, "adam1")
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    with torch.no_grad():
        logits = module(batch, 0)
    out = dict(sd)
    out.update(grads)
    out.update(after)
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), genre=genre.numpy(), tags=tags.numpy(),
                    logits=logits[:, :16 if suffix else L].numpy(), loss=loss.detach().numpy(), emb_out=hooks["emb_out"].numpy(),
                    enc_out=hooks["enc_out"].numpy(),
                    logits_head=np.int64(16 if suffix else L),
                    cfg=np.array([B, L, d, h, N, V, len(gtok), len(ttok)]), lr=np.float32(1e-3),
                    betas=np.array([0.99, 0.998], np.float32)))
    np.savez_compressed(os.path.join(HERE, f"kebert4rec_{variant}{suffix}.npz"), **out)
    print("kebert4rec", variant + suffix, float(loss))


def gen_ubert4rec(variant: str, B=4, L=10, d=32, h=2, N=2, NI=43, NG=7, NU=6, K=3, lengths=(10, 7, 4, 2), suffix=""):
    """ubert4rec: UBERTMaskedTrainingModule + UBERT4RecModel (the user-attribute model): a user token prepended to
    the item sequence, attribute embeddings, optional segment embedding, causal transformer (bidirectional=False)
    core/models/ubert4rec/ubert4rec_model.py:16-92, components.py:13-203, core/modules/ubert_masked_training_module.py"""
    tok = S.make_tokenizer(NI)
    gtok = S.make_tokenizer(NG, "Genre")
    utok = S.make_tokenizer(NU, "User")
    S.set_context({"item": tok, "genre": gtok, "user": utok})
    from asme.core.models.ubert4rec.ubert4rec_model import UBERT4RecModel
    from asme.core.modules.ubert_masked_training_module import UBERTMaskedTrainingModule
    V = len(tok)
    if variant == "seg":
        additional = {"genre": {"embedding_type": "content_embedding"}}
        users = {"user": {"embedding_type": "user_embedding"}}
        segment = True
    else:
        additional = {"genre": {"embedding_type": "linear_upscale"}}
        users = {"user": {"embedding_type": "user_linear_upscale"}}
        segment = False
    torch.manual_seed(10)
    # UBERT4RecModel / UBERTMaskedTrainingModule carry the Inject* annotations without @inject: pass them
    model = UBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                           item_vocab_size=V, max_seq_length=L, transformer_dropout=0.0,
                           additional_attributes=additional,
                           additional_tokenizers={"tokenizers.genre": gtok, "tokenizers.user": utok},
                           user_attributes=users, positional_embedding=True, segment_embedding=segment)
    module = UBERTMaskedTrainingModule(model=model, item_tokenizer=tok, metrics=None, num_warmup_steps=0)
    sd = _sd(model)
    g = torch.Generator().manual_seed(11)
    lengths = list(lengths)
    seq, tgt = _cloze_batch(g, B, L, V, lengths)
    if variant == "seg":
        genre = torch.randint(3, len(gtok), (B, L), generator=g)
        genre[seq == PAD] = PAD
        user = torch.randint(3, len(utok), (B, L), generator=g)   # the user id in every column; column 0 is read
    else:
        genre = torch.randint(3, len(gtok), (B, L, K), generator=g)
        genre[:, :, 2][torch.rand(B, L, generator=g) < 0.5] = 0
        genre[seq == PAD] = 0
        user = torch.randint(3, len(utok), (B, L, K), generator=g)
        user[:, :, 1] = 0                                          # a pad category the user upscaler does count
    batch = {"item": seq, "item.target": tgt, "genre": genre, "user": user}
    res = module.training_step(batch, 0)
    loss = res["loss"]
    loss.backward()
    grads = _grads(model)
    opts = module.configure_optimizers()
    opts[0].step()
    after = _params(model, "adam1")
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    ev = seq.clone()
    ev[ev == MASK] = 7
    for b, n in enumerate(lengths):
        ev[b, n - 1] = MASK
    with torch.no_grad():
        logits = module(batch, 0)
        pred = module.predict_step(dict(batch, item=ev), 0)
    out = dict(sd)
    out.update(grads)
    out.update(after)
    head = 16 if suffix else logits.shape[1]
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), genre=genre.numpy(), user=user.numpy(),
                    logits=logits[:, :head].numpy(), loss=loss.detach().numpy(), eval_seq=ev.numpy(),
                    eval_logits=pred.numpy(), logits_head=np.int64(head),
                    cfg=np.array([B, L, d, h, N, V, len(gtok), len(utok)]), lr=np.float32(1e-3),
                    betas=np.array([0.99, 0.998], np.float32)))
    np.savez_compressed(os.path.join(HERE, f"ubert4rec_{variant}{suffix}.npz"), **out)
    print("ubert4rec", variant + suffix, float(loss), logits.shape)


def gen_narm():
    """narm: NextItemPredictionTrainingModule + NarmModel (single-target CE)
    core/models/narm/narm_model.py:25-68, components.py:14-56, layers.py:8-120, core/losses/losses.py:65-115"""
    B, L, E, H, NI = 5, 9, 16, 24, 39
    tok = S.make_tokenizer(NI)
    S.set_context({"item": tok})
    from asme.core.models.narm.narm_model import NarmModel
    from asme.core.modules.next_item_prediction_training_module import NextItemPredictionTrainingModule
    V = len(tok)
    torch.manual_seed(8)
    model = NarmModel(item_embedding_size=E, global_encoder_size=H, global_encoder_num_layers=1,
                      embedding_dropout=0.0, context_dropout=0.0)
    module = NextItemPredictionTrainingModule(model=model, metrics=None)
    sd = _sd(model)
    g = torch.Generator().manual_seed(9)
    lengths = [9, 7, 4, 2, 1]
    seq = _ragged_batch(g, B, L, V, lengths)
    tgt = torch.randint(3, V, (B,), generator=g)
    res = module.training_step({"item": seq, "item.target": tgt}, 0)
    loss = res["loss"]
    loss.backward()
    grads = _grads(model)
    opt = module.configure_optimizers()
    opt.step()
    after = _params(model, "adam1")
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    with torch.no_grad():
        logits = module({"item": seq}, 0)
    out = dict(sd)
    out.update(grads)
    out.update(after)
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), logits=logits.numpy(), loss=loss.detach().numpy(),
                    cfg=np.array([B, L, E, H, V]), lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32)))
    np.savez_compressed(os.path.join(HERE, "narm.npz"), **out)
    print("narm", float(loss))


def _ddp_round(build, sd, slices, W):
    """One Lightning-DDP step over W ranks, restated serially (the reference's multi-GPU training,
    configs/ml-20m/unfiltered/sasrec_config.jsonnet:77-79, bert4rec_config.jsonnet:83-87): every rank starts from
    the same parameters (DDP's broadcast), runs training_step on ITS slice (its own mean loss), backward; the
    gradients are averaged over the ranks (DDP's all-reduce / W); every rank takes the same optimizer step.
    Returns (per-rank losses, averaged gradients, parameters after the step)."""
    losses, avg = [], None
    for r in range(W):
        model, module = build()
        model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
        loss = module.training_step(slices[r], 0)["loss"]
        loss.backward()
        losses.append(float(loss))
        g = {n: (p.grad.detach().clone() if p.grad is not None else torch.zeros_like(p))
             for n, p in model.named_parameters()}
        avg = g if avg is None else {n: avg[n] + g[n] for n in avg}
    avg = {n: v / W for n, v in avg.items()}
    model, module = build()
    model.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in sd.items()})
    for n, p in model.named_parameters():
        p.grad = avg[n].clone()
    opts = module.configure_optimizers()
    opt = opts if isinstance(opts, torch.optim.Optimizer) else opts[0]
    opt = opt[0] if isinstance(opt, (list, tuple)) else opt
    opt.step()
    return (np.array(losses, np.float32), {n: v.numpy() for n, v in avg.items()},
            {n: p.detach().numpy().copy() for n, p in model.named_parameters()})


# ragged lengths of the 16 DDP sequences: every slice of 2 (W = 8) and of 8 (W = 2) has its own token count, so the
# per-rank mean losses differ from the global mean
_DDP_LENGTHS = (50, 43, 37, 31, 25, 50, 12, 8, 50, 3, 17, 29, 44, 6, 1, 38)


def gen_ddp_sasrec(worlds=(2, 8), B=16, L=50, d=128, h=2, N=2, NI=300, lengths=_DDP_LENGTHS):
    """sasrec-neg under DDP (BASELINE C4's semantics; the row-sharded table must reproduce them):
    SequenceNextItemPredictionTrainingModule + SASRecModel at the production widths (d = 128, h = 2, d_ff = 512),
    L = 50, ragged sessions; per W: each rank's loss, the rank-averaged gradients, the parameters after one Adam step
    core/modules/sequence_next_item_prediction_training_module.py:73-115,181-185, core/losses/sasrec/sas_rec_losses.py"""
    tok = S.make_tokenizer(NI)
    S.set_context({"item": tok})
    from asme.core.models.sasrec.sasrec_model import SASRecModel
    from asme.core.modules.sequence_next_item_prediction_training_module import \
        SequenceNextItemPredictionTrainingModule
    V = len(tok)

    def build():
        model = SASRecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                            max_seq_length=L, transformer_dropout=0.0)
        return model, SequenceNextItemPredictionTrainingModule(model=model, metrics=None)

    torch.manual_seed(20)
    sd = _sd(build()[0])
    g = torch.Generator().manual_seed(21)
    full = _ragged_batch(g, B, L + 1, V, [n + 1 for n in lengths])
    seq, pos = full[:, :L].clone(), full[:, 1:].clone()
    for b, n in enumerate(lengths):
        seq[b, n:] = PAD
        pos[b, n:] = PAD
    neg = torch.randint(3, V, (B, L), generator=g)
    neg[seq == PAD] = PAD
    out = dict(sd)
    for W in worlds:
        per = B // W
        slices = [{"item": seq[r * per:(r + 1) * per], "positive_samples": pos[r * per:(r + 1) * per],
                   "negative_samples": neg[r * per:(r + 1) * per]} for r in range(W)]
        losses, avg, after = _ddp_round(build, sd, slices, W)
        out[f"w{W}/loss"] = losses
        out.update({f"w{W}/grad/{n}": v for n, v in avg.items()})
        out.update({f"w{W}/adam1/{n}": v for n, v in after.items()})
        print(f"ddp sasrec W={W} losses", losses)
    out.update(dict(seq=seq.numpy(), pos=pos.numpy(), neg=neg.numpy(), worlds=np.array(worlds),
                    cfg=np.array([B, L, d, h, N, V]), lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32),
                    weight_decay=np.float32(1e-3)))
    np.savez_compressed(os.path.join(HERE, "ddp_sasrec_neg.npz"), **out)


def gen_ddp_kebert4rec(worlds=(2, 8), B=16, L=50, d=128, h=2, N=2, NI=300, NG=7, NT=9, K=3, lengths=_DDP_LENGTHS):
    """KeBERT4Rec (post-fusion genre, pre-fusion tags) under DDP (BASELINE C5): MaskedTrainingModule at the production
    widths, L = 50, ragged cloze batches (each rank's masked mean over its own masked positions); per W: each rank's
    loss, the rank-averaged gradients, the parameters after one Adam step
    core/models/kebert4rec/kebert4rec_model.py:24-89, core/modules/masked_training_module.py:93-111,167-189"""
    tok = S.make_tokenizer(NI)
    gtok = S.make_tokenizer(NG, "Genre")
    ttok = S.make_tokenizer(NT, "Tag")
    S.set_context({"item": tok, "genre": gtok, "tags": ttok})
    from asme.core.models.kebert4rec.kebert4rec_model import KeBERT4RecModel
    from asme.core.modules.masked_training_module import MaskedTrainingModule
    V = len(tok)

    def build():
        model = KeBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                                max_seq_length=L, transformer_dropout=0.0,
                                prefusion_attributes={"tags": {"embedding_type": "linear_upscale"}},
                                postfusion_attributes={"genre": {"embedding_type": "content_embedding"}})
        return model, MaskedTrainingModule(model=model, metrics=None, num_warmup_steps=0)

    torch.manual_seed(22)
    sd = _sd(build()[0])
    g = torch.Generator().manual_seed(23)
    seq, tgt = _cloze_batch(g, B, L, V, list(lengths))
    genre = torch.randint(3, NG + 3, (B, L), generator=g)
    tags = torch.randint(3, NT + 3, (B, L, K), generator=g)
    tags[:, :, 2][torch.rand(B, L, generator=g) < 0.5] = 0
    genre[seq == PAD] = PAD
    tags[seq == PAD] = 0
    out = dict(sd)
    for W in worlds:
        per = B // W
        slices = [{"item": seq[r * per:(r + 1) * per], "item.target": tgt[r * per:(r + 1) * per],
                   "genre": genre[r * per:(r + 1) * per], "tags": tags[r * per:(r + 1) * per]} for r in range(W)]
        losses, avg, after = _ddp_round(build, sd, slices, W)
        out[f"w{W}/loss"] = losses
        out.update({f"w{W}/grad/{n}": v for n, v in avg.items()})
        out.update({f"w{W}/adam1/{n}": v for n, v in after.items()})
        print(f"ddp kebert4rec W={W} losses", losses)
    out.update(dict(seq=seq.numpy(), target=tgt.numpy(), genre=genre.numpy(), tags=tags.numpy(),
                    worlds=np.array(worlds), cfg=np.array([B, L, d, h, N, V, len(gtok), len(ttok)]),
                    lr=np.float32(1e-3), betas=np.array([0.99, 0.998], np.float32)))
    np.savez_compressed(os.path.join(HERE, "ddp_kebert4rec_post.npz"), **out)


def gen_metrics():
    """NDCG/recall/MRR via the reference metric classes (core/metrics/*.py) + AllItemsSampler."""
    from asme.core.metrics.ndcg import NormalizedDiscountedCumulativeGainMetric
    from asme.core.metrics.recall import RecallMetric
    from asme.core.metrics.mrr import MRRMetric
    from asme.core.metrics.container.metrics_sampler import AllItemsSampler
    g = torch.Generator().manual_seed(11)
    B, V = 64, 300
    logits = torch.randn(B, V, generator=g)
    targets = torch.randint(0, V, (B,), generator=g)
    # make some targets rank high so the @k values are non-trivial
    for b in range(0, B, 3):
        logits[b, targets[b]] = logits[b].max() + 0.01 * (b % 7 + 1)  # strictly above: tie-free
    samp = AllItemsSampler().sample(None, targets, logits)
    out = {"logits": logits.numpy(), "targets": targets.numpy()}
    for k in (1, 5, 10):
        for name, cls in (("ndcg", NormalizedDiscountedCumulativeGainMetric), ("recall", RecallMetric)):
            m = cls(k=k)
            m.update(samp.sampled_predictions, samp.positive_item_mask, samp.metric_mask)
            out[f"{name}@{k}"] = m.compute().numpy()
            out[f"{name}@{k}/per_row"] = m._calc_metric(samp.sampled_predictions, samp.positive_item_mask,
                                                        torch.ones_like(samp.positive_item_mask)).numpy()
    m = MRRMetric(k=10)
    m.update(samp.sampled_predictions, samp.positive_item_mask, samp.metric_mask)
    out["mrr@10"] = m.compute().numpy()
    np.savez_compressed(os.path.join(HERE, "metrics.npz"), **out)
    print("metrics", {k: float(v) for k, v in out.items() if "@" in k and "/" not in k})


def _markov_sessions(rng, n_users, n_items, min_len, max_len):
    """Synthetic ml-1m-shaped interaction sequences with learnable structure: a sparse
    random Markov chain over a Zipf-popular item catalogue (ids 3..3+n_items-1)."""
    pop = 1.0 / np.arange(1, n_items + 1) ** 0.8
    pop /= pop.sum()
    succ = rng.choice(n_items, size=(n_items, 8), p=pop)
    seqs = []
    for _ in range(n_users):
        n = int(rng.integers(min_len, max_len + 1))
        s = [int(rng.choice(n_items, p=pop))]
        for _ in range(n - 1):
            s.append(int(succ[s[-1], rng.integers(0, 8)]) if rng.random() < 0.7 else int(rng.choice(n_items, p=pop)))
        seqs.append(np.array(s, np.int64) + 3)
    return seqs


def gen_ml1m_anchor(train_steps: int = 400):
    """ml-1m-shaped NDCG@10 parity anchor: train the reference SASRec-neg on a
    synthetic 6,040-user / 3,416-item set with the reference module for `train_steps` steps,
    then evaluate NDCG@10 (AllItemsSampler, full catalogue) on each user's held-out last item."""
    rng = np.random.default_rng(1234)
    n_users, n_items, L, d = 6040, 3416, 50, 64
    tok = S.make_tokenizer(n_items)
    S.set_context({"item": tok})
    from asme.core.models.sasrec.sasrec_model import SASRecModel
    from asme.core.modules.sequence_next_item_prediction_training_module import \
        SequenceNextItemPredictionTrainingModule
    from asme.core.metrics.ndcg import NormalizedDiscountedCumulativeGainMetric
    from asme.core.metrics.container.metrics_sampler import AllItemsSampler
    V = len(tok)
    seqs = _markov_sessions(rng, n_users, n_items, 20, 120)
    torch.manual_seed(42)
    model = SASRecModel(transformer_hidden_size=d, num_transformer_heads=2, num_transformer_layers=2,
                        max_seq_length=L, transformer_dropout=0.2)
    module = SequenceNextItemPredictionTrainingModule(model=model, metrics=None)
    opt = module.configure_optimizers()
    torch.set_num_threads(8)
    model.train()
    g = torch.Generator().manual_seed(77)
    B = 128
    for step in range(train_steps):
        idx = rng.integers(0, n_users, B)
        seq = torch.zeros(B, L, dtype=torch.long)
        pos = torch.zeros(B, L, dtype=torch.long)
        for r, u in enumerate(idx):
            s = seqs[u][:-1][-(L + 1):]          # train on everything but the held-out last item
            n = len(s) - 1
            seq[r, :n] = torch.from_numpy(s[:-1])
            pos[r, :n] = torch.from_numpy(s[1:])
        neg = torch.randint(3, V, (B, L), generator=g)
        neg[seq == PAD] = PAD
        opt.zero_grad()
        loss = module.training_step({"item": seq, "positive_samples": pos, "negative_samples": neg}, step)["loss"]
        loss.backward()
        opt.step()
        if step % 100 == 0:
            print("  anchor train step", step, float(loss))
    torch.set_num_threads(1)
    model.eval()
    eval_seq = np.zeros((n_users, L), np.int16)
    targets = np.zeros(n_users, np.int64)
    for u, s in enumerate(seqs):
        inp = s[:-1][-L:]
        eval_seq[u, :len(inp)] = inp
        targets[u] = s[-1]
    metric = NormalizedDiscountedCumulativeGainMetric(k=10)
    per_user = []
    with torch.no_grad():
        for i in range(0, n_users, 256):
            seq = torch.from_numpy(eval_seq[i:i + 256].astype(np.int64))
            tg = torch.from_numpy(targets[i:i + 256])
            pred = module.predict_step({"item": seq}, 0)
            samp = AllItemsSampler().sample(seq, tg, pred)
            metric.update(samp.sampled_predictions, samp.positive_item_mask, samp.metric_mask)
            per_user.append(metric._calc_metric(samp.sampled_predictions, samp.positive_item_mask,
                                                torch.ones_like(samp.positive_item_mask)).numpy())
    ndcg = metric.compute()
    out = {f"sd/{k}": v.detach().numpy() for k, v in model.state_dict().items()
           if not k.startswith("_projection_layer.")}     # projection keys alias the embedding module
    out.update(dict(eval_seq=eval_seq, targets=targets, ndcg10=ndcg.numpy(), ndcg10_per_user=np.concatenate(per_user),
                    cfg=np.array([n_users, L, d, 2, 2, V])))
    np.savez_compressed(os.path.join(HERE, "ml1m_anchor.npz"), **out)
    print("ml1m anchor NDCG@10 =", float(ndcg))


def gen_bert4rec_anchor(train_steps: int = 300):
    """BERT4Rec NDCG@10 parity anchor through the masked evaluation: the reference BERT4Rec (tied head) trained with
    the reference MaskedTrainingModule on the ml-1m-shaped synthetic sessions of gen_ml1m_anchor (cloze masking
    p = 0.2 plus the last item, torch generator draws), evaluated as ASME evaluates it: each user's sequence without
    its held-out last item, a MASK appended (LastItemMaskProcessor, data/datasets/processors/last_item_mask.py:35-44),
    predictions at the MASK (masked_training_module.py:80-91), AllItemsSampler + NDCG@10 (core/metrics)."""
    rng = np.random.default_rng(1234)
    n_users, n_items, L, d = 6040, 3416, 50, 64
    tok = S.make_tokenizer(n_items)
    S.set_context({"item": tok})
    from asme.core.models.bert4rec.bert4rec_model import BERT4RecModel
    from asme.core.modules.masked_training_module import MaskedTrainingModule
    from asme.core.metrics.ndcg import NormalizedDiscountedCumulativeGainMetric
    from asme.core.metrics.container.metrics_sampler import AllItemsSampler
    V = len(tok)
    seqs = _markov_sessions(rng, n_users, n_items, 20, 120)
    torch.manual_seed(43)
    model = BERT4RecModel(transformer_hidden_size=d, num_transformer_heads=2, num_transformer_layers=2,
                          max_seq_length=L, transformer_dropout=0.1)
    module = MaskedTrainingModule(model=model, metrics=None, num_warmup_steps=0)
    opts = module.configure_optimizers()
    opt = opts[0] if isinstance(opts, (list, tuple)) else opts
    opt = opt[0] if isinstance(opt, (list, tuple)) else opt
    torch.set_num_threads(8)
    model.train()
    g = torch.Generator().manual_seed(78)
    B = 128
    for step in range(train_steps):
        idx = rng.integers(0, n_users, B)
        seq = torch.zeros(B, L, dtype=torch.long)
        for r, u in enumerate(idx):
            s = seqs[u][:-1][-L:]                # train on everything but the held-out last item
            seq[r, :len(s)] = torch.from_numpy(s)
        valid = seq != PAD
        m = (torch.rand(B, L, generator=g) < 0.2) & valid
        last = valid.sum(1) - 1
        m[torch.arange(B), last] = True
        tgt = torch.where(m, seq, torch.zeros_like(seq))
        inp = torch.where(m, torch.full_like(seq, MASK), seq)
        opt.zero_grad()
        loss = module.training_step({"item": inp, "item.target": tgt}, step)["loss"]
        loss.backward()
        opt.step()
        if step % 100 == 0:
            print("  bert4rec anchor train step", step, float(loss))
    torch.set_num_threads(1)
    model.eval()
    eval_seq = np.zeros((n_users, L), np.int16)
    targets = np.zeros(n_users, np.int64)
    for u, s in enumerate(seqs):
        inp = s[:-1][-(L - 1):]
        eval_seq[u, :len(inp)] = inp
        eval_seq[u, len(inp)] = MASK                 # the last-item mask appended
        targets[u] = s[-1]
    metric = NormalizedDiscountedCumulativeGainMetric(k=10)
    per_user = []
    with torch.no_grad():
        for i in range(0, n_users, 256):
            seq = torch.from_numpy(eval_seq[i:i + 256].astype(np.int64))
            tg = torch.from_numpy(targets[i:i + 256])
            pred = module.predict_step({"item": seq}, 0)
            samp = AllItemsSampler().sample(seq, tg, pred)
            metric.update(samp.sampled_predictions, samp.positive_item_mask, samp.metric_mask)
            per_user.append(metric._calc_metric(samp.sampled_predictions, samp.positive_item_mask,
                                                torch.ones_like(samp.positive_item_mask)).numpy())
    ndcg = metric.compute()
    out = {f"sd/{k}": v.detach().numpy() for k, v in model.state_dict().items()}
    out.update(dict(eval_seq=eval_seq, targets=targets, ndcg10=ndcg.numpy(), ndcg10_per_user=np.concatenate(per_user),
                    cfg=np.array([n_users, L, d, 2, 2, V])))
    np.savez_compressed(os.path.join(HERE, "bert4rec_anchor.npz"), **out)
    print("bert4rec anchor NDCG@10 =", float(ndcg))


if __name__ == "__main__":
    which = sys.argv[1:] or ["models", "metrics", "ml1m"]
    if "models" in which:
        gen_sasrec_neg()
        gen_sasrec_cross()
        gen_bert4rec("transpose_embedding")
        gen_bert4rec("linear")
        gen_kebert4rec("pre")
        gen_kebert4rec("post")
        gen_narm()
    if "ubert4rec" in which or "models" in which:
        gen_ubert4rec("seg")
        gen_ubert4rec("upscale")
    if "d128" in which:
        # the benchmarked composition: d = 128, h = 2, d_ff = 4d = 512, L = 200 -- every
        # Linear on the weight-stationary GEMM, the fused FFN, the production weight-gradient shapes
        big = dict(B=4, L=200, d=128, h=2, N=2, NI=1000, suffix="_d128")
        gen_sasrec_neg(lengths=(200, 173, 61, 7), **big)
        gen_bert4rec("linear", lengths=(200, 150, 37, 5), adam2=False, **big)
        gen_bert4rec("transpose_embedding", lengths=(200, 150, 37, 5), adam2=False, **big)
        gen_kebert4rec("post", lengths=(200, 120, 77, 9), NG=7, NT=9, K=3, **big)
    if "d128b" in which:
        # the same composition for the other model families (round 3): vocabularies of 300 items keep the
        # fixtures small; d, h, d_ff and L are the production ones
        big = dict(B=4, L=200, d=128, h=2, N=2, NI=300, suffix="_d128")
        gen_sasrec_cross(lengths=(200, 143, 40, 6), **big)
        gen_kebert4rec("pre", lengths=(200, 131, 57, 8), NG=7, NT=9, K=3, **big)
        gen_ubert4rec("seg", lengths=(200, 160, 33, 4), NG=7, NU=6, K=3, **big)
        gen_ubert4rec("upscale", lengths=(200, 97, 21, 3), NG=7, NU=6, K=3, **big)
    if "ddp" in which:
        # multi-GPU semantics (BASELINE C4 / C5): Lightning DDP over W = 2 and 8 ranks, restated serially
        gen_ddp_sasrec()
        gen_ddp_kebert4rec()
    if "bert4rec_anchor" in which:
        gen_bert4rec_anchor()
    if "metrics" in which:
        gen_metrics()
    if "ml1m" in which:
        gen_ml1m_anchor()
