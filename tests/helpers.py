"""Fixture loading / model construction shared by the tests."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def state_dict(z):
    return {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}


def prefixed(z, prefix):
    n = len(prefix) + 1
    return {k[n:]: z[k] for k in z.files if k.startswith(prefix + "/")}


class Tok:
    """tokenizer stand-in for the models' attribute vocabularies (len only)"""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


def base_name(name):
    """fixture name without its shape suffix (sasrec_neg_d128 -> sasrec_neg)"""
    return name[:-5] if name.endswith("_d128") else name


def build_model(asme, name, z):
    cfg = [int(x) for x in z["cfg"]]
    name = base_name(name)
    if name == "sasrec_neg" or name == "sasrec_cross":
        B, L, d, h, N, V = cfg
        return asme.SASRecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                                item_vocab_size=V, max_seq_length=L, transformer_dropout=0.0,
                                mode="neg_sampling" if name == "sasrec_neg" else "full")
    if name.startswith("bert4rec"):
        B, L, d, h, N, V = cfg
        kind = "transpose_embedding" if "transpose" in name else "linear"
        return asme.BERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                                  item_vocab_size=V, max_seq_length=L, transformer_dropout=0.0,
                                  project_layer_type=kind)
    if name.startswith("kebert4rec"):
        B, L, d, h, N, V, VG, VT = cfg
        toks = {"tokenizers.genre": Tok(VG), "tokenizers.tags": Tok(VT)}
        if name.endswith("pre"):
            pre = {"genre": {"embedding_type": "content_embedding"}, "tags": {"embedding_type": "linear_upscale"}}
            post = None
        else:
            pre = {"tags": {"embedding_type": "linear_upscale"}}
            post = {"genre": {"embedding_type": "content_embedding"}}
        return asme.KeBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                                    item_vocab_size=V, max_seq_length=L, transformer_dropout=0.0,
                                    prefusion_attributes=pre, postfusion_attributes=post,
                                    additional_attributes_tokenizer=toks)
    if name.startswith("ubert4rec"):
        B, L, d, h, N, V, VG, VU = cfg
        toks = {"tokenizers.genre": Tok(VG), "tokenizers.user": Tok(VU)}
        if name.endswith("seg"):
            add, users = {"genre": {"embedding_type": "content_embedding"}}, {"user": {"embedding_type": "user_embedding"}}
        else:
            add = {"genre": {"embedding_type": "linear_upscale"}}
            users = {"user": {"embedding_type": "user_linear_upscale"}}
        return asme.UBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=h, num_transformer_layers=N,
                                   item_vocab_size=V, max_seq_length=L, transformer_dropout=0.0,
                                   additional_attributes=add, additional_tokenizers=toks, user_attributes=users,
                                   positional_embedding=True, segment_embedding=name.endswith("seg"))
    if name == "narm":
        B, L, E, H, V = cfg
        return asme.NarmModel(item_vocab_size=V, item_embedding_size=E, global_encoder_size=H,
                              global_encoder_num_layers=1, embedding_dropout=0.0, context_dropout=0.0)
    raise KeyError(name)


MODEL_FIXTURES = ["sasrec_neg", "sasrec_cross", "bert4rec_transpose_embedding", "bert4rec_linear",
                  "kebert4rec_pre", "kebert4rec_post", "ubert4rec_seg", "ubert4rec_upscale", "narm"]
# the benchmarked composition: d = 128, h = 2, d_ff = 512, L = 200 (make_golden.py d128)
D128_FIXTURES = ["sasrec_neg_d128", "bert4rec_linear_d128", "bert4rec_transpose_embedding_d128",
                 "kebert4rec_post_d128", "sasrec_cross_d128", "kebert4rec_pre_d128", "ubert4rec_seg_d128",
                 "ubert4rec_upscale_d128"]


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def close(a, b, rtol=1e-3, atol=1e-7):
    """max|a-b| <= rtol * max|b| + atol (atol covers gradients that are analytically zero, e.g. the
    key-projection bias, where both sides are rounding noise)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max()) <= rtol * float(np.abs(b).max()) + atol


ADAM_EPS = 1e-8


def elem_excess(got, ref, rtol=1e-3, floor=1e-3):
    """max over elements of |got - ref| / (rtol * (|ref| + floor * max|ref|)): <= 1 passes (the element-wise criterion
    of test_gpu_elementwise.py: each element within rtol of its own magnitude; entries more than three decades below
    the tensor's scale, where fp32 summation order alone decides the low bits, get an absolute floor)"""
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if ref.size == 0:
        return 0.0
    scale = np.abs(ref).max()
    if scale == 0.0:
        return 0.0 if np.abs(got).max() == 0.0 else float("inf")
    return float((np.abs(got - ref) / (rtol * (np.abs(ref) + floor * scale))).max())


def adam_excess(got, want, g, lr, rtol=1e-3, floor=1e-3):
    """element-wise excess of a parameter after Adam's first step, lr * g / (|g| + eps) with g the total gradient
    (weight decay included): the parameter's own element-wise bound plus what the gradient's element-wise bound
    (rtol * (|g| + floor * max|g|), the one the gradients are held to) moves the update by -- its derivative
    lr * eps / (|g| + eps)^2 is large only for |g| within a few decades of eps, where fp32 summation order alone
    decides the gradient's low bits"""
    got, want, g = (np.asarray(x, np.float64) for x in (got, want, g))
    if want.size == 0:
        return 0.0
    ag = np.abs(g)
    tol = rtol * (np.abs(want) + floor * np.abs(want).max()) + \
        lr * ADAM_EPS / (ag + ADAM_EPS) ** 2 * rtol * (ag + floor * ag.max())
    err = np.abs(got - want)
    with np.errstate(divide="ignore", invalid="ignore"):  # (a zero bound passes only an exact match)
        return float(np.where(err == 0, 0.0, err / tol).max())


def ddp_errors(z, world, rank, loss, grads, params, tables=(), rows=None):
    """element-wise excess of one rank's DDP step against a make_golden.py `ddp` fixture: its loss (w{W}/loss[rank]),
    the rank-averaged gradients (w{W}/grad/*; None entries are not checked) and the parameters after the Adam step
    (w{W}/adam1/*).  Names in `tables` are row shards: compared against rows rank::W of the fixture's table (`rows`:
    the shard's row count)."""
    errs = {"loss": abs(loss - float(z[f"w{world}/loss"][rank])) / (1e-4 * abs(float(z[f"w{world}/loss"][rank])))}
    for n, ref in prefixed(z, f"w{world}/grad").items():
        if n.endswith("attention.linear_layers.1.bias"):
            continue  # analytically zero: both sides are rounding noise
        gref = ref[rank::world] if n in tables else ref
        if grads.get(n) is not None:
            errs["grad/" + n] = elem_excess(grads[n], gref)
        want = z[f"w{world}/adam1/{n}"]
        p0 = z["sd/" + n]
        if n in tables:
            want, p0 = want[rank::world], p0[rank::world]
        wd = float(z["weight_decay"]) if "weight_decay" in z.files else 0.0
        errs["adam1/" + n] = adam_excess(params[n], want, gref + wd * p0, float(z["lr"]))
    return errs
