"""NARM training step at the ml-1m configuration (configs-new/narm/ml-1m.yaml: batch 128, L = 200, E = 64, H = 128,
|V| = 3706, dropout 0.2 / 0.2) on the hand kernels (NextItemPredictionTrainingModule + NarmModel + FusedAdam) beside
the reference's PyTorch formulation of the same step on the same GPU (pack_padded_sequence + nn.GRU on MIOpen,
torch local encoder, B(E_items) bilinear head, nn.CrossEntropyLoss, torch.optim.Adam;
core/models/narm/components.py:32-56, layers.py:32-120).  Prints one JSON line.

    python tools/narm_bench.py [--batch 128] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402


class TorchNarm(nn.Module):
    """the reference's NARM forward in stock PyTorch ops (timing comparison only)"""

    def __init__(self, V, E, H, p_emb, p_ctx):
        super().__init__()
        self.emb = nn.Embedding(V, E)
        self.drop = nn.Dropout2d(p_emb)
        self.gru = nn.GRU(E, H, batch_first=True)
        self.A1 = nn.Linear(H, H, bias=False)
        self.A2 = nn.Linear(H, H, bias=False)
        self.v = nn.Parameter(torch.rand(H) * 2 - 1)
        self.ctx_drop = nn.Dropout(p_ctx)
        self.B = nn.Linear(E, 2 * H, bias=False)

    def forward(self, seq):
        mask = seq.ne(0)
        x = self.drop(self.emb(seq))
        lengths = mask.sum(-1).cpu()
        packed = nn.utils.rnn.pack_padded_sequence(x, lengths, batch_first=True, enforce_sorted=False)
        h_i, h_t = self.gru(packed)
        c_g = h_t[-1]
        h_i, _ = nn.utils.rnn.pad_packed_sequence(h_i, batch_first=True, total_length=seq.shape[1])
        proj = torch.sigmoid(self.A1(c_g).unsqueeze(1) + self.A2(h_i))
        alphas = torch.matmul(proj, self.v).unsqueeze(2)
        c_l = (mask.unsqueeze(-1).to(h_i.dtype) * (alphas * h_i)).sum(1)
        c = self.ctx_drop(torch.cat([c_g, c_l], 1))
        items = self.drop(self.emb(torch.arange(self.emb.num_embeddings, device=seq.device)))
        return c @ self.B(items).t()


def batch(B, L, V, dev, g):
    lengths = torch.randint(1, L + 1, (B,), generator=g)
    seq = torch.randint(3, V, (B, L), generator=g)
    seq[torch.arange(L).unsqueeze(0) >= lengths.unsqueeze(1)] = 0
    return seq.to(dev), torch.randint(3, V, (B,), generator=g).to(dev)


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq-len", type=int, default=200)
    ap.add_argument("--items", type=int, default=3706)
    ap.add_argument("--emb", type=int, default=64)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    dev = torch.device("cuda:0")
    B, L, V, E, H = a.batch, a.seq_len, a.items, a.emb, a.hidden
    g = torch.Generator().manual_seed(0)
    batches = [batch(B, L, V, dev, g) for _ in range(8)]

    model = asme.NarmModel(item_vocab_size=V, item_embedding_size=E, global_encoder_size=H,
                           global_encoder_num_layers=1, embedding_dropout=0.2, context_dropout=0.2).to(dev)
    module = asme.NextItemPredictionTrainingModule(model=model, item_tokenizer=asme.tokenization.Tokenizer(V - 3),
                                                   metrics=None)
    opt = module.configure_optimizers()
    it = [0]

    def ours():
        seq, tgt = batches[it[0] % 8]
        it[0] += 1
        asme.modules.train_step(module, opt, None, {"item": seq, "item.target": tgt}, 0)

    ref = TorchNarm(V, E, H, 0.2, 0.2).to(dev)
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3, betas=(0.99, 0.998))

    def theirs():
        seq, tgt = batches[it[0] % 8]
        it[0] += 1
        loss = F.cross_entropy(ref(seq), tgt, ignore_index=0)
        loss.backward()
        ropt.step()
        ropt.zero_grad(set_to_none=True)

    t_ours = timed(ours, a.steps, a.warmup)
    t_ref = timed(theirs, a.steps, a.warmup)
    print(json.dumps({"workload": "narm ml-1m train step", "batch": B, "seq_len": L, "items": V, "emb": E,
                      "hidden": H, "ms_per_step": round(t_ours * 1e3, 3), "seq_per_s": round(B / t_ours, 1),
                      "torch_reference_ms_per_step": round(t_ref * 1e3, 3),
                      "torch_reference_seq_per_s": round(B / t_ref, 1), "speedup": round(t_ref / t_ours, 2)}))


if __name__ == "__main__":
    main()
