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
