"""Headline benchmark: SASRec-neg training sequences/sec at B=1024/GPU, L=200, |I|=10M, d=128 (BASELINE.json).

One step = forward + backward + FusedAdam over every parameter (the dense Adam over all 10,000,003 item
rows included, reference semantics SURVEY Q7) on one synthetic batch that is already resident in HBM.
    python bench.py                      # N=1, defaults finish in a few minutes
    torchrun --nproc-per-node N bench.py --gpus N
Prints ONE JSON line (rank 0).  See DESIGN.md §Measurement for the roofline accounting.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import platform
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP32_MFMA_TFS = 157.3  # dense fp32 MFMA spec
# kernels that compute their fp32 products as six bf16 MFMAs of split operands (csrc/common.h, bf16x6): their
# ceiling is the dense bf16 MFMA peak (2516.6 TF/s = 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz) over 6
PEAK_BF16X6_TFS = 2516.6 / 6
BF16X6_KERNELS = {"asme_ws_linear", "asme_linear_weight_grad", "asme_linear_xent_fwd", "asme_linear_xent_bwd",
                  "asme_linear_xent_fwd_dh", "asme_linear_xent_bwd_dw", "asme_logits", "asme_catalog_rank_x6",
                  "asme_catalog_count_above_x6"}


def instrumented_steps(steps):
    """timed steps whose C-ABI calls carry HIP start/stop events for the per-kernel rooflines: the last two.
    The events cost ~2 us of device time each (~0.25 ms per step with every timed kernel bracketed, measured
    with --kernel-events off), so bracketing every step would understate the step rate by ~3 %."""
    return min(steps, 2)


def mfma_peak(name):
    return round(PEAK_BF16X6_TFS, 1) if name in BF16X6_KERNELS else PEAK_FP32_MFMA_TFS


def committed_profile(name, config):
    """a committed PMC summary under profiles/ (JSON with "config"), when it was taken at this exact configuration"""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        j = json.load(f)
    return j if j.get("config") == config else {}


def gemm_work(T, d, ffn, fused_o=False):
    """algorithmic work per launch of the transformer's GEMM calls.  Per block: the forward QKV
    (d -> 3d), O (d -> d), FFN in (d -> ffn, its epilogue writing the activation and the factor keep * GELU'(pre) the
    backward needs in place of the pre-activation) and FFN out (ffn -> d), and the same four shapes as input
    gradients (the GELU one reading the factor), 8 asme_ws_linear calls: bytes in units of T x 4 B = 2 (8d + 3 ffn);
    the four weight gradients on asme_linear_weight_grad: dY + X = 8d + 2 ffn.  fused_o: the O projection's forward
    runs as asme_ws_linear_residual_ln (X and the residual in, s and LN(s) out + the row statistics), the other 7
    calls per block on asme_ws_linear"""
    wg_flops = 2.0 * T * (3 * d * d + d * d + ffn * d + d * ffn)
    ws_bytes = 2 * T * 4.0 * (8 * d + 3 * ffn)
    wg_bytes = T * 4.0 * (8 * d + 2 * ffn)
    out = {"asme_ws_linear": ("gemm", 2 * wg_flops / 8, ws_bytes / 8),
           "asme_linear_weight_grad": ("gemm", wg_flops / 4, wg_bytes / 4)}
    if fused_o:
        o_flops, o_bytes = 2.0 * T * d * d, T * 4.0 * 2 * d
        out["asme_ws_linear"] = ("gemm", (2 * wg_flops - o_flops) / 7, (ws_bytes - o_bytes) / 7)
        out["asme_ws_linear_residual_ln"] = ("gemm", o_flops, T * 4.0 * 4 * d + T * 8)
    return out


def fused_o_projection(asme, d):
    """the transformer's O projection runs fused with its residual + pre-LN (layers.TransformerLayer)"""
    return bool(asme.layers.TransformerLayer.fuse_output_projection) and d == 128


def roofline_entries(kstats, work, traffic, busy=None):
    """one roofline per timed C-ABI call.  work[name] = (bound, amount) or ("gemm", flops, bytes): a GEMM's bound is
    read off its arithmetic intensity against the ridge of its MFMA ceiling and the HBM peak (the transformer's
    tall-skinny Linear GEMMs, 38-48 FLOP/B, sit below the bf16x6 ridge of 52 FLOP/B: HBM-bound)"""
    out = []
    for name, st in kstats.items():
        if not st["count"] or name not in work:
            continue
        w = work[name]
        secs = st["avg_ms"] / 1e3
        extra = {}
        if w[0] == "gemm":
            flops, nbytes = w[1], w[2]
            ai = flops / nbytes
            ridge = mfma_peak(name) * 1e12 / (PEAK_HBM_GBS * 1e9)
            bound, amount = ("mfma", flops) if ai >= ridge else ("hbm", nbytes)
            extra = {"flop_per_byte": round(ai, 2), "ridge_flop_per_byte": round(ridge, 2),
                     "mfma_tflops": round(flops / secs / 1e12, 2), "mfma_peak": mfma_peak(name),
                     "mfma_frac": round(flops / secs / 1e12 / mfma_peak(name), 4),
                     "flops_per_launch": flops, "bytes_per_launch": nbytes}
        else:
            bound, amount = w
            extra = {("flops_per_launch" if bound == "mfma" else "bytes_per_launch"): amount}
        if bound == "mfma":
            ach, peak, unit = amount / secs / 1e12, mfma_peak(name), "TFLOP/s"
        else:
            ach, peak, unit = amount / secs / 1e9, PEAK_HBM_GBS, "GB/s"
        if busy and name in busy:  # PMC: fraction of all SIMD cycles with the matrix pipe busy (MFMA utilisation)
            extra["mfma_busy"] = busy[name]
        if bound == "hbm" and amount / secs / 1e9 > PEAK_HBM_GBS:
            extra["note"] = ("above the HBM peak: part of the algorithmic bytes is served from the L2 / the 256 MB "
                             "Infinity Cache (rows read in slot order from the step's staged rows)")
        out.append({"kernel": name, "bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                    "frac": round(ach / peak, 4), "traffic": traffic.get(name), "avg_ms": round(st["avg_ms"], 4),
                    "launches": st["count"], "total_ms": round(st["total_ms"], 3), **extra})
    out.sort(key=lambda r: -r["total_ms"])
    return out


# the north_star's named kernel targets (BASELINE.json): >= 70 % of the HBM roofline on the embedding gather,
# >= 50 % MFMA on the logits GEMM -- surfaced by name in the compact line
TARGET_KERNELS = ("asme_embedding_ln_fwd", "asme_embedding_ln_bwd", "asme_linear_xent_fwd_dh",
                  "asme_linear_xent_bwd_dw", "asme_catalog_rank_x6", "asme_catalog_count_above_x6")
ROOF_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "avg_ms", "launches")


def slim_roofline(r):
    if not r:
        return r
    out = {k: r[k] for k in ROOF_KEYS if k in r}
    for k in ("mfma_busy", "mfma_frac"):
        if k in r:
            out[k] = r[k]
    return out


def compact(result, top=3):
    """The one stdout line: the contract keys, the dominant kernel's roofline, the CPU baseline, the top-`top`
    rooflines and the named target kernels of every workload -- short enough that the driver's stdout tail holds
    all of it (the full record goes to --full-json)."""
    out = {k: v for k, v in result.items() if k not in ("rooflines", "workloads", "eval", "cpu_baseline")}
    out["roofline"] = slim_roofline(result.get("roofline"))
    rl = result.get("rooflines") or []
    out["rooflines_top"] = [slim_roofline(r) for r in rl[:top]]
    targets = {r["kernel"]: r["frac"] for r in rl if r["kernel"] in TARGET_KERNELS}
    cb = result.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
        if "single_thread" in cb:
            out["cpu_baseline"]["single_thread"] = cb["single_thread"]["value"]
    else:
        out["cpu_baseline"] = None
    if result.get("eval"):
        e = result["eval"]
        out["eval"] = {k: e[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "ndcg@10") if k in e}
        out["eval"]["roofline"] = slim_roofline(e.get("roofline"))
        targets.update({r["kernel"]: r["frac"] for r in e.get("rooflines", []) if r["kernel"] in TARGET_KERNELS})
    wl = {}
    for name, w in (result.get("workloads") or {}).items():
        c = {k: w[k] for k in ("value", "unit", "ms_per_step", "n_gpus") if k in w}
        c["parallelism"] = w.get("config", {}).get("parallelism")
        cbw = w.get("cpu_baseline")
        c["cpu_baseline"] = ({k: cbw[k] for k in ("value", "cores", "kind", "batch", "s_per_step") if k in cbw}
                             if cbw else None)
        wrl = w.get("rooflines") or []
        c["rooflines_top"] = [{k: r[k] for k in ("kernel", "bound", "frac", "achieved", "unit", "avg_ms") if k in r}
                              for r in wrl[:top]]
        tw = {r["kernel"]: r["frac"] for r in wrl if r["kernel"] in TARGET_KERNELS}
        if tw:
            c["target_kernels"] = tw
        wl[name] = c
    if wl:
        out["workloads"] = wl
    out["target_kernels"] = targets
    return out


def emit(result, args):
    """rank 0: the full record to --full-json, the compact line to stdout"""
    if args.full_json:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.full_json)), exist_ok=True)
            with open(args.full_json, "w") as f:
                json.dump(result, f, indent=1)
        except OSError as e:
            print(f"bench.py: could not write {args.full_json}: {e}", file=sys.stderr, flush=True)
    print(json.dumps(compact(result)), flush=True)


def parse(argv=None):
    return build_parser().parse_args(argv)


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["sasrec-neg", "bert4rec", "kebert4rec"], default="sasrec-neg",
                    help="sasrec-neg: the headline (BASELINE C4 at N=1); bert4rec: BASELINE C3, cloze-masked BERT4Rec "
                         "with the full-catalogue softmax (--items 27000), batches built by the GPU cloze producer; "
                         "kebert4rec: BASELINE C5 (--items 13000), a synthetic per-item category side attribute")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="sequences per GPU")
    ap.add_argument("--seq-len", type=int, default=200)
    ap.add_argument("--items", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--heads", type=int, default=2)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--dropout", type=float, default=0.2)
    ap.add_argument("--table-grad", choices=["sparse", "dense"], default="sparse")
    ap.add_argument("--main-stream", choices=["default", "high"], default="default",
                    help="run the training steps on a high-priority stream (producer side streams keep the default)")
    ap.add_argument("--ids-ahead", choices=["on", "mid", "off"], default="on",
                    help="SASRec (unsharded): produce the next batch and its table-id dedup / occurrence CSR on a "
                         "side stream during the current step (off: inline, the A/B form)")
    ap.add_argument("--ids", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--kernel-events", choices=["on", "off"], default="on",
                    help="HIP events around the timed kernels (off: no per-kernel rooflines; for A/B of their cost)")
    ap.add_argument("--producer", choices=["resident", "gpu"], default="gpu",
                    help="gpu (default): every step samples a fresh batch from sessions in HBM with the GPU pos/neg "
                         "sampler (asme_posneg_sample) inside the timed step; resident: two pre-built device batches "
                         "alternating (rows touched one or two steps earlier: less lazy catch-up per step)")
    ap.add_argument("--legs", default="bert4rec:27000,kebert4rec:13000,sasrec_zipf,sasrec_overlap",
                    help="with the sasrec-neg headline: the other BASELINE workloads run in the same invocation and "
                         "reported under \"workloads\" of the one JSON line (name:items, comma-separated; "
                         "C3 BERT4Rec |I| = 27,000, C5 KeBERT4Rec |I| = 13,000, sasrec_zipf: the headline step on "
                         "Zipf(1.07) ids at the headline's --items (SURVEY §8d secondary); 'none' to skip)")
    ap.add_argument("--eval-steps", type=int, default=8,
                    help="timed full-catalogue evaluation batches (one validation pass, one catalogue split) of the "
                         "trained headline model (0: no eval leg)")
    ap.add_argument("--eval-warmup", type=int, default=1)
    ap.add_argument("--full-json", default=os.path.join("gpurun_out", "bench_full.json"),
                    help="where rank 0 writes the full record (every roofline of every workload); stdout carries the "
                         "compact line ('' to skip the file)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle leg (rank 0, N=1)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend for N>1 (nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    ap.add_argument("--sharded", action="store_true",
                    help="run the row-sharded path even at N=1 (1-rank RCCL group): its overhead without the fabric")
    ap.add_argument("--cpu-batch", type=int, default=0, help="sequences per CPU-baseline step (0: --batch)")
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--cpu-batch-1t", type=int, default=16, help="sequences of the single-thread CPU step")
    ap.add_argument("--cpu-batch-masked", type=int, default=64,
                    help="sequences per CPU-baseline step of the BERT4Rec / KeBERT4Rec workloads")
    ap.add_argument("--sampler-sessions", type=int, default=16, help="sessions for the CPU sampler rate")
    return ap


def parse_legs(spec: str):
    if not spec or spec == "none":
        return []
    out = []
    for part in spec.split(","):
        name, _, items = part.partition(":")
        if name not in ("bert4rec", "kebert4rec", "sasrec_zipf", "sasrec_overlap"):
            raise SystemExit(f"--legs: unknown workload {name!r}")
        out.append((name, int(items) if items else {"bert4rec": 27000, "kebert4rec": 13000, "sasrec_zipf": 0,
                                                    "sasrec_overlap": 0}[name]))
    return out


def session_ids(n, V, g, kind):
    """n item ids in [3, V) for the synthetic sessions: uniform, or Zipf(1.07) over item rank (id 3 the most popular;
    inverse CDF of the continuous power law, SURVEY §8d secondary)"""
    if kind == "uniform":
        return torch.randint(3, V, (n,), device=g.device, generator=g)
    u = torch.rand(n, device=g.device, generator=g, dtype=torch.float64)
    a, m = 1.07, V - 3
    hmax = (m ** (1 - a) - 1) / (1 - a)
    r = ((u * hmax) * (1 - a) + 1) ** (1 / (1 - a))
    return r.long().clamp(1, m) + 2


def synthetic_batch(B, L, V, seed, dev, kind="uniform"):
    """Full-length sequences (no padding): ids ~ U[3, V) (or Zipf(1.07) over item rank), pos = next id,
    neg ~ U[3, V)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    full = session_ids(B * (L + 1), V, g, kind).view(B, L + 1)
    g2 = torch.Generator(device=dev).manual_seed(seed + 1)
    neg = torch.randint(3, V, (B, L), device=dev, generator=g2)
    return {"item": full[:, :L].contiguous(), "positive_samples": full[:, 1:].contiguous(), "negative_samples": neg}


def cpu_share() -> int:
    """host threads this job may use: the scheduler affinity, capped by OMP_NUM_THREADS when the pool sets it
    (on the GPU box os.cpu_count() reports the whole machine, many times this job's share)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def cpu_model_name() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "cpu"


def cpu_baseline(args, V):
    """CPU restatement (oracle/asme_oracle.py, reference op order) timed on the host cores, SURVEY §8(d): the same
    step (fwd + bwd + dense torch Adam over the full 10M-row table) on the same B = 1024 batch shape, all of this
    job's threads, --cpu-warmup warm-up + --cpu-steps timed steps; then the single-thread rate (same model and
    optimizer state, a --cpu-batch-1t batch) and the reference CPU input pipeline's rate (the pos/neg sampler's
    0/1-weight multinomial over |V| per session, pos_neg_sampler.py:41-106)."""
    from oracle import asme_oracle as O
    threads = cpu_share()
    torch.set_num_threads(threads)
    d, L, N, h = args.dim, args.seq_len, args.layers, args.heads
    sd = O.init_sasrec_state(V, L, d, N, seed=0)
    params = [p.requires_grad_(True) for p in sd.values()]
    opt = torch.optim.Adam(params, lr=1e-3, betas=(0.99, 0.998), weight_decay=1e-3, foreach=False)
    B = args.cpu_batch or args.batch

    def run(batch_size, n_warm, n_timed, tag):
        batch = synthetic_batch(batch_size, L, V, 1234, torch.device("cpu"))
        times = []
        for i in range(n_warm + n_timed):
            t0 = time.perf_counter()
            O.sasrec_neg_train_step(sd, opt, batch["item"], batch["positive_samples"], batch["negative_samples"], h,
                                    dropout=args.dropout)
            times.append(time.perf_counter() - t0)
            print(f"[cpu_baseline] {tag} step {i + 1}/{n_warm + n_timed}: {times[-1]:.2f} s", file=sys.stderr,
                  flush=True)
        return sum(times[n_warm:]) / n_timed

    per_step = run(B, args.cpu_warmup, args.cpu_steps, f"B={B} x{threads} threads")
    torch.set_num_threads(1)
    B1 = args.cpu_batch_1t
    per_step_1t = run(B1, 0, 1, f"B={B1} x1 thread")
    torch.set_num_threads(threads)
    # the reference's CPU negative sampler at this |V| (one DataLoader worker = one core)
    g = torch.Generator().manual_seed(1235)
    sessions = torch.randint(3, V, (args.sampler_sessions, L + 1), generator=g).tolist()
    torch.set_num_threads(1)
    t0 = time.perf_counter()
    for sess in sessions:
        O.pos_neg(sess, V, (0, 1, 2))
    sampler = len(sessions) / (time.perf_counter() - t0)
    torch.set_num_threads(threads)
    return {"value": round(B / per_step, 3), "unit": "sequences/s", "cores": threads, "kind": "port",
            "batch": B, "s_per_step": round(per_step, 3),
            "single_thread": {"value": round(B1 / per_step_1t, 3), "batch": B1, "s_per_step": round(per_step_1t, 3)},
            "input_pipeline": {"value": round(sampler, 2), "unit": "sessions/s per core",
                               "what": f"reference pos/neg sampler (torch.multinomial over |V|={V}), L={L}"},
            "machine_cpus": os.cpu_count(),
            "sample": f"SASRec-neg fwd+bwd+dense Adam, B={B} L={L} d={d} |V|={V} (full table), {args.cpu_steps} "
                      f"timed steps after {args.cpu_warmup} warm-up, {per_step:.2f} s/step on {threads} threads "
                      f"(this job's CPU share; the machine has {os.cpu_count()}), torch CPU fp32, {cpu_model_name()}"}


def cpu_baseline_masked(args, model, V, kebert, n_genre, workload):
    """CPU restatement (oracle/asme_oracle.py bert4rec_logits / kebert4rec_logits, reference op order) of the C3 / C5
    step timed on the host cores: the model's own initial parameters (reference state_dict keys) copied to the CPU,
    the reference's full (B, L, |V|) logits + CrossEntropyLoss(ignore_index) (masked_training_module.py:93-111),
    backward, torch.optim.Adam; dropout off.  A bounded sample: --cpu-batch-masked sequences of a 20 % cloze
    batch (the full-catalogue logits, linear in B, dominate), --cpu-warmup + --cpu-steps steps."""
    from oracle import asme_oracle as O
    threads = cpu_share()
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()
          if v.dtype.is_floating_point}
    opt = torch.optim.Adam(list(sd.values()), lr=1e-3, betas=(0.9, 0.999), foreach=False)
    B, L = args.cpu_batch_masked, args.seq_len
    g = torch.Generator().manual_seed(4321)
    seq = torch.randint(3, V, (B, L), generator=g)
    masked = torch.rand(B, L, generator=g) < 0.2
    target = torch.where(masked, seq, torch.zeros_like(seq))
    inp = torch.where(masked, torch.ones_like(seq), seq)
    genre = torch.where(inp > 0, seq % (n_genre - 1) + 1, 0)
    times = []
    for i in range(args.cpu_warmup + args.cpu_steps):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        if kebert:
            logits = O.kebert4rec_logits(sd, inp, args.heads, {"genre": (genre, "content_embedding", n_genre)}, {})
        else:
            logits = O.bert4rec_logits(sd, inp, args.heads, tied=True)
        loss = O.cross_entropy(logits.reshape(-1, logits.shape[-1]), target.reshape(-1))
        loss.backward()
        opt.step()
        times.append(time.perf_counter() - t0)
        print(f"[cpu_baseline] {workload} B={B} step {i + 1}/{args.cpu_warmup + args.cpu_steps}: "
              f"{times[-1]:.2f} s", file=sys.stderr, flush=True)
    per_step = sum(times[args.cpu_warmup:]) / args.cpu_steps
    name = "KeBERT4Rec" if kebert else "BERT4Rec"
    return {"value": round(B / per_step, 3), "unit": "sequences/s", "cores": threads, "kind": "port", "batch": B,
            "s_per_step": round(per_step, 3), "machine_cpus": os.cpu_count(),
            "sample": f"{name} cloze fwd+bwd+Adam, B={B} L={L} |V|={V} (full (B, L, |V|) logits + CE, as the "
                      f"reference), {args.cpu_steps} timed steps after {args.cpu_warmup} warm-up, "
                      f"{per_step:.2f} s/step on {threads} threads, torch CPU fp32, dropout off, {cpu_model_name()}"}


def bench_bert4rec(args, asme, dev, world, rank, workload, items):
    """BASELINE config C3: BERT4Rec (tied head), cloze masking p = 0.2 / last-item-only 0.1, B per GPU, full
    catalogue CE over |V| = items + 3 (C5: KeBERT4Rec with a category side attribute).  Every step builds its
    batch on the GPU (collate + asme_cloze_mask) from sessions in HBM inside the timed region; data parallel over
    ranks (dataparallel.GradientAllReduce: bucketed RCCL all-reduce overlapped with the backward).  Returns the
    leg's result (rank 0 prints it, alone or inside the headline line's "workloads")."""
    V = items + 3
    B, L, d = args.batch, args.seq_len, args.dim
    kebert = workload == "kebert4rec"
    n_genre = 64  # synthetic side attribute: category of the item, content_embedding
    with torch.device(dev):
        if kebert:
            model = asme.KeBERT4RecModel(transformer_hidden_size=d, num_transformer_heads=args.heads,
                                         num_transformer_layers=args.layers, item_vocab_size=V, max_seq_length=L,
                                         transformer_dropout=args.dropout,
                                         prefusion_attributes={"genre": {"embedding_type": "content_embedding"}},
                                         additional_attributes_tokenizer={
                                             "tokenizers.genre": asme.tokenization.Tokenizer(n_genre - 3)})
        else:
            model = asme.BERT4RecModel(transformer_hidden_size=d, num_transformer_heads=args.heads,
                                       num_transformer_layers=args.layers, item_vocab_size=V, max_seq_length=L,
                                       transformer_dropout=args.dropout)
    tok = asme.tokenization.Tokenizer(items)
    module = asme.MaskedTrainingModule(model=model, item_tokenizer=tok, metrics=None)
    module.train()
    opt, sched = asme.modules.split_optimizers(module.configure_optimizers())
    n_sess = max(4 * B, 8192)
    g = torch.Generator(device=dev).manual_seed(4321 + rank)
    flat = torch.randint(3, V, (n_sess * L,), device=dev, generator=g)
    store = asme.batches.SessionStore(flat, torch.arange(n_sess + 1, device=dev) * L)
    cloze = asme.batches.ClozeMaskProcessor(tok, 0.2, 0.1)
    order = torch.randperm(n_sess, device=dev, generator=g)

    # N > 1: data parallel with DDP semantics (dataparallel.GradientAllReduce: bucketed RCCL all-reduce launched
    # from the backward hooks, the row-sparse item table reduced last)
    reducer = None
    if world > 1:
        reducer = asme.dataparallel.GradientAllReduce(module)
        reducer.broadcast_parameters(module)

    # each step's batch is produced on a side stream one step ahead, and its masked rows selected there
    # (module.prefetch: torch.nonzero's host read waits for the side stream only) once the current step is enqueued
    side = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)

    def make_batch(i):
        with torch.cuda.stream(side):
            idx = order[(i * B) % (n_sess - B + 1):][:B]
            items, lengths = asme.batches.padded_session_batch(store, idx, L)
            b = cloze.process_batch(items, lengths, seed=1000 + i)
            if kebert:
                b["genre"] = torch.where(items > 0, items % (n_genre - 1) + 1, 0)
        return b

    ahead = {}

    def step(i):
        batch = ahead.pop(i, None) or make_batch(i)
        main.wait_stream(side)  # the batch and its prefetched rows
        for t in list(batch.values()) + list(module._rows_ahead[1:] if module._rows_ahead else []):
            t.record_stream(main)
        nxt = ahead[i + 1] = make_batch(i + 1)
        if reducer is not None:
            asme.dataparallel.train_step(module, opt, sched, reducer, batch, i)
        else:
            asme.modules.train_step(module, opt, sched, batch, i)
        with torch.cuda.stream(side):
            module.prefetch(nxt)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    timer = asme._lib.KernelTimer(["asme_attention_fwd", "asme_attention_bwd", "asme_ws_linear",
                                   "asme_ws_linear_residual_ln", "asme_linear_weight_grad", "asme_cross_entropy_fwd",
                                   "asme_cross_entropy_bwd",
                                   "asme_linear_xent_fwd", "asme_linear_xent_bwd", "asme_linear_xent_fwd_dh",
                                   "asme_linear_xent_bwd_dw", "asme_cloze_mask",
                                   "asme_residual_ln_fwd", "asme_residual_ln_bwd", "asme_embedding_fwd",
                                   "asme_embedding_bwd"])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        with timer if i >= args.steps - instrumented_steps(args.steps) else contextlib.nullcontext():
            step(args.warmup + i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    T, H, dk = B * L, args.heads, d // args.heads
    pairs = B * H * L * L  # bidirectional
    ffn = 4 * d
    M = 0.9 * 0.2 * T + 0.1 * B  # expected non-ignored rows of a cloze batch
    work = {"asme_attention_fwd": ("mfma", 4.0 * pairs * dk), "asme_attention_bwd": ("mfma", 10.0 * pairs * dk),
            **gemm_work(T, d, ffn, fused_o_projection(asme, d)),
            "asme_linear_xent_fwd": ("mfma", 2.0 * M * V * d), "asme_linear_xent_bwd": ("mfma", 4.0 * M * V * d),
            # training form: the forward computes the logits and dH (both algorithmic), the backward dW (its logits
            # recompute is not counted)
            "asme_linear_xent_fwd_dh": ("mfma", 4.0 * M * V * d), "asme_linear_xent_bwd_dw": ("mfma", 2.0 * M * V * d),
            "asme_cross_entropy_fwd": ("hbm", M * V * 4.0), "asme_cross_entropy_bwd": ("hbm", 2 * M * V * 4.0),
            "asme_residual_ln_fwd": ("hbm", 4 * T * d * 4 + T * 8),
            "asme_residual_ln_bwd": ("hbm", 5 * T * d * 4 + T * 8),
            "asme_embedding_fwd": ("hbm", T * 8 + 2 * T * d * 4 + T * 16),
            "asme_embedding_bwd": ("hbm", T * 8 + 3 * T * d * 4 + T * 16)}
    lb = committed_profile("logits_mfma_busy.json", {"workload": workload, "rows": 36966, "items": V, "dim": d})
    # HBM traffic per launch from the committed rocprofv3 PMC pass over this workload (tools/pmc_traffic.py)
    tp = committed_profile(f"pmc_traffic_{workload}.json", {"batch": B, "seq_len": L, "items": items,
                                                              "dim": d, "layers": args.layers})
    rooflines = roofline_entries(timer.summary(), work, tp.get("bytes_per_launch", {}),
                                 lb.get("mfma_busy") if B == 1024 and L == 200 else None)
    name = "KeBERT4Rec" if kebert else "BERT4Rec"
    result = {"metric": f"training sequences/sec ({name} cloze, B={B} L={L} |V|={V}, fwd+bwd+Adam)",
              "value": round(B * world * args.steps / elapsed, 2), "unit": "sequences/s", "n_gpus": world,
              "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
              "data": "synthetic sessions, GPU cloze masking inside the step, random-init weights",
              "config": {"workload": ("kebert4rec cloze train step (BASELINE C5)" if kebert
                                      else "bert4rec cloze train step (BASELINE C3)"), "model": name,
                         "global_batch": B * world, "batch_per_gpu": B, "seq_len": L, "items": items,
                         "dim": d, "heads": H, "layers": args.layers, "dropout": args.dropout,
                         "fused_xent": asme.modules.FUSED_XENT, "parallelism": f"dp{world}"},
              "roofline": rooflines[0] if rooflines else None, "rooflines": rooflines, "cpu_baseline": None}
    if rank == 0 and world == 1 and args.cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_masked(args, model, V, kebert, n_genre, workload)
    if reducer is not None:
        reducer.remove()
    return result


def bench_eval(args, asme, dev, world, rank, module, get_batch, ids_kind):
    """Full-catalogue evaluation of the trained SASRec at |I| = args.items: B sequences per GPU,
    each scored against EVERY item of the catalogue (the reference's AllItemsSampler + argsort, sasrec/components.py:
    46-61, metrics/common.py:4-27) and its target ranked without materialising the (B, |I|) scores -- one step =
    the eval-mode transformer forward + asme_catalog_rank_x6 (at N > 1: every rank counts the items of its shard above
    every rank's targets, asme_catalog_count_above, + one all_reduce of the int32 counts) + NDCG@10 / recall@10 from
    the ranks.  The timed region is one validation pass of --eval-steps batches: its first batch splits the frozen
    catalogue into the bf16 planes (asme_catalog_split, 2.3 ms at |I| = 10M), the others reuse them (ops.CatalogPlanes,
    as a validation epoch does).  Same contract as the training legs: warm-up, barrier + synchronize around exactly
    --eval-steps."""
    B, L, d, V = args.batch, args.seq_len, args.dim, args.items + 3
    module.eval()
    ndcg = asme.metrics.NormalizedDiscountedCumulativeGainMetric(10)
    recall = asme.metrics.RecallMetric(10)
    batches = []
    for j in range(2):
        b = get_batch(10_000 + j)
        batches.append({"item": b["item"], "item.target": b["positive_samples"][:, -1].contiguous()})

    def step(i):
        with torch.no_grad():
            ranks = module.catalog_ranks(batches[i % 2])
            ndcg.update_ranks(ranks)
            recall.update_ranks(ranks)

    for i in range(args.eval_warmup):
        step(i)
    ndcg.reset()
    recall.reset()
    module._catalog_planes.clear()  # the timed pass makes its own catalogue split
    timer = asme._lib.KernelTimer(["asme_catalog_rank_x6", "asme_catalog_count_above_x6", "asme_catalog_split",
                                   "asme_catalog_target_scores_x6", "asme_ws_linear", "asme_ws_linear_residual_ln",
                                   "asme_attention_fwd",
                                   "asme_embedding_ln_fwd"])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.eval_steps):
        with timer if i >= args.eval_steps - instrumented_steps(args.eval_steps) else contextlib.nullcontext():
            step(i)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    module.train()
    nq = B * world  # every rank scores all ranks' queries against its 1/W of the catalogue at N > 1
    scan = 2.0 * nq * V * d / world
    # the ranking scan: 2 nq |I| d FLOP per step (the target-score pass's 2 nq d is negligible; the catalogue split,
    # 5.1 GB in -> 7.7 GB of planes out, is an HBM pass of its own)
    work = {"asme_catalog_rank_x6": ("mfma", scan), "asme_catalog_count_above_x6": ("mfma", scan),
            "asme_catalog_split": ("hbm", (V // world) * d * (4.0 + 6.0)), **gemm_work(B * L, d, 4 * d, fused_o_projection(asme, d))}
    rooflines = roofline_entries(timer.summary(), work, {})
    return {"metric": f"evaluation sequences/sec (SASRec full-catalogue rank + NDCG@10, B={B} L={L} |I|={args.items})",
            "value": round(B * world * args.eval_steps / elapsed, 2), "unit": "sequences/s",
            "ms_per_step": round(1000 * elapsed / args.eval_steps, 3), "steps": args.eval_steps,
            "warmup": args.eval_warmup, "ids": ids_kind,
            "ndcg@10": round(float(ndcg.compute()), 6), "recall@10": round(float(recall.compute()), 6),
            "roofline": rooflines[0] if rooflines else None, "rooflines": rooflines}


def bench_sasrec(args, asme, dev, world, rank, ids_kind, with_eval=True, overlap=False):
    """The SASRec-neg training step (BASELINE C2 / C4): B sequences per GPU, |I| = args.items, the GPU pos/neg
    producer inside the timed step; ids_kind "uniform" (the headline) or "zipf" (Zipf(1.07) over item rank, seed
    1234: SURVEY §8d's secondary, hot keys for the dedup / occurrence CSR / ordered reduce-apply).  Returns the result
    dict (rank 0 prints it as the headline line, or inside it under "workloads")."""
    V = args.items + 3
    B, L, d = args.batch, args.seq_len, args.dim
    torch.manual_seed(rank)
    sharded = world > 1 or args.sharded
    # N > 1: the item table is row-sharded over the ranks (RCCL all-to-all of ids / rows / row grads,
    # one all_reduce of the replicated dense gradients); N = 1: the whole table on the one GPU
    rows = asme.sharded.shard_rows(V, world, rank) if sharded else V
    with torch.device(dev):
        model = asme.SASRecModel(transformer_hidden_size=d, num_transformer_heads=args.heads,
                                 num_transformer_layers=args.layers, item_vocab_size=rows, max_seq_length=L,
                                 transformer_dropout=args.dropout)
    tok = asme.tokenization.Tokenizer(args.items)
    if sharded:
        module = asme.sharded.ShardedSequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok,
                                                                              metrics=None, vocab=V,
                                                                              overlap_negatives=overlap)
        module.broadcast_dense_parameters()
        step_fn = None  # set below: each step also starts the next batch's id routing (module.prefetch)
    else:
        module = asme.SequenceNextItemPredictionTrainingModule(model=model, item_tokenizer=tok, metrics=None,
                                                               table_grad=args.table_grad)
        step_fn = lambda b, i: asme.modules.train_step(module, opt, None, b, i)  # noqa: E731
    module.train()
    opt = module.configure_optimizers()
    batches = [synthetic_batch(B, L, V, 1234 + 7 * (rank * 2 + i), dev, ids_kind) for i in range(2)]
    if args.producer == "gpu":
        # sessions of L + 1 items in HBM; each step's batch (x, pos, sampled negatives) is built on the GPU
        # inside the step (asme_posneg_sample), as the reference's DataLoader would produce it
        n_sess = max(4 * B, 8192)
        g = torch.Generator(device=dev).manual_seed(4321 + rank)
        flat = session_ids(n_sess * (L + 1), V, g, ids_kind)
        store = asme.batches.SessionStore(flat, torch.arange(n_sess + 1, device=dev) * (L + 1))
        sampler = asme.batches.PositiveNegativeSamplerProcessor(tok)
        order = torch.randperm(n_sess, device=dev, generator=g)

        def get_batch(i):
            idx = order[(i * B) % (n_sess - B + 1):][:B]
            b = sampler.process_batch(store, idx, L, seed=1000 + i)
            return {k: b[k] for k in ("item", "positive_samples", "negative_samples")}
    else:
        def get_batch(i):
            return batches[i % 2]

    if sharded:
        ahead = {}

        def batch_at(j):
            b = ahead.pop(j, None)
            return b if b is not None else get_batch(j)

        last = args.warmup + args.steps - 1

        def step_fn(b_unused, i, j=None):  # j: absolute batch index (warm-up i, timed warmup + i)
            cur = batch_at(j)
            nxt = None
            if j < last and j != args.warmup - 1:  # (no prefetch across the warm-up / timed boundary)
                nxt = ahead[j + 1] = get_batch(j + 1)
            asme.sharded.train_step(module, opt, cur, i, next_batch=nxt)

        def run(j, i):
            step_fn(None, i, j)
    elif args.producer == "gpu" and args.ids_ahead != "off":
        # the next batch is produced on a side stream during this step -- the pos / neg sampler, then the id-only
        # half of its table plan (dedup + occurrence CSR, module.prefetch -> ops.TableIdsAhead) -- the way the masked
        # legs produce theirs; the step's training_step waits for it.  No prefetch across the warm-up / timed
        # boundary or past the last timed step: the timed region produces and applies exactly K batches.
        side = torch.cuda.Stream(dev)
        ahead = {}
        last = args.warmup + args.steps - 1

        def produce_next(j):
            if j < last and j != args.warmup - 1:
                with torch.cuda.stream(side):
                    nb = ahead[j + 1] = get_batch(j + 1)
                    module.prefetch(nb)

        def run(j, i):
            b = ahead.pop(j, None)
            if b is None:
                b = get_batch(j)
            if args.ids_ahead == "mid":  # (A/B form: the side work enqueued after this step's forward)
                loss = module.training_step(b, i)["loss"]
                produce_next(j)
                asme.modules.backward(loss)
                opt.step()
                opt.zero_grad(set_to_none=True)
                return
            step_fn(b, i)
            produce_next(j)
    else:
        def run(j, i):
            step_fn(get_batch(j), i)

    for i in range(args.warmup):
        run(i, i)
    # the warm-up steps' own deferred zero-gradient table updates are applied before the timer starts, so the timed
    # region holds exactly K steps of optimizer work: the steps' staged rows plus the end-of-run flush of every row's
    # remaining timed steps (otherwise the timed region also replayed W steps of warm-up updates for every row)
    opt.flush()
    torch.cuda.synchronize()

    # per-kernel device time of the dominant kernel (HIP events on the launching stream)
    timer = asme._lib.KernelTimer([] if args.kernel_events == "off" else [
                                   "asme_adam_rows_step", "asme_attention_fwd", "asme_attention_bwd",
                                   "asme_embedding_fwd", "asme_embedding_bwd", "asme_embedding_ln_fwd",
                                   "asme_embedding_ln_bwd", "asme_lazy_adam_catch_up",
                                   "asme_lazy_adam_apply", "asme_lazy_adam_stage", "asme_lazy_adam_apply_staged",
                                   "asme_sampled_logits_fwd", "asme_sampled_logits_bwd", "asme_gelu_dropout_fwd", "asme_gelu_dropout_bwd",
                                   "asme_linear_weight_grad", "asme_residual_ln_fwd", "asme_residual_ln_bwd",
                                   "asme_ws_linear", "asme_ws_linear_residual_ln", "asme_posneg_sample",
                                   "asme_table_grad_reduce_apply",
                                   "asme_dedup_ids", "asme_dedup_ids_segments", "asme_occurrence_csr",
                                   "asme_position_grad", "asme_reduce_rows", "asme_sasrec_bce_fwd",
                                   "asme_sasrec_bce_bwd"])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last_unique = []
    _orig_release = asme.ops.SparseTablePlan.release

    def _release(plan):  # record the unique-row count of the step (for the byte accounting)
        if plan.dim and not last_unique:
            last_unique.append(plan.count)  # (read after the timed region: no host sync inside it)
        _orig_release(plan)

    asme.ops.SparseTablePlan.release = _release
    host_s = []  # host time to issue each step (no synchronisation inside a step): a CPU-bound step shows ~= ms_per_step
    for i in range(args.steps):
        h0 = time.perf_counter()
        with timer if i >= args.steps - instrumented_steps(args.steps) else contextlib.nullcontext():
            run(args.warmup + i, i)
        host_s.append(time.perf_counter() - h0)
    # lazily deferred zero-gradient Adam updates of the item table are part of the work: apply them all
    # (exact dense-Adam state) inside the timed region, timed on its own
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record()
    opt.flush()
    f1.record()
    torch.cuda.synchronize()
    flush_ms = f0.elapsed_time(f1)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / args.steps
    value = B * world * args.steps / elapsed

    kstats = timer.summary()
    asme.ops.SparseTablePlan.release = _orig_release
    eval_leg = (bench_eval(args, asme, dev, world, rank, module, get_batch, ids_kind)
                if args.eval_steps > 0 and with_eval else None)
    U = int(last_unique[0].item()) if last_unique else min(3 * B * L, V)
    # distinct rows the sampled head gathers (positive and negative ids of a step's batch): the head's compulsory
    # row bytes -- each further occurrence of a row is served from the L2 / MALL, not re-fetched from HBM
    lb = get_batch(args.warmup + args.steps - 1) if not sharded else None
    U_pn = (int(torch.unique(torch.cat([lb["positive_samples"].reshape(-1), lb["negative_samples"].reshape(-1)]))
                .numel()) if lb is not None else 2 * B * L)
    T = B * L
    H, dk = args.heads, d // args.heads
    ffn = 4 * d
    # algorithmic work per launch.  Attention: causal pairs only (L(L+1)/2 per head), the
    # forward = 2 matmul passes (QK^T, PV), the backward = 5 (recomputed S, dP, dV, dK in the dK/dV pass, which
    # stores dS; dQ = dS K) -- the kernels execute exactly these.
    pairs = B * H * L * (L + 1) / 2.0
    work = {
        "asme_attention_fwd": ("mfma", 2 * 2.0 * pairs * dk),
        "asme_attention_bwd": ("mfma", 5 * 2.0 * pairs * dk),
        # the GEMM calls per block, averaged per launch (gemm_work)
        **gemm_work(T, d, ffn, fused_o_projection(asme, d)),
        "asme_gelu_dropout_fwd": ("hbm", 2 * T * ffn * 4),
        "asme_residual_ln_fwd": ("hbm", 4 * T * d * 4 + T * 8),
        "asme_residual_ln_bwd": ("hbm", 5 * T * d * 4 + T * 8),
        "asme_embedding_fwd": ("hbm", T * 8 + 2 * T * d * 4 + T * 16),
        "asme_embedding_bwd": ("hbm", T * 8 + 3 * T * d * 4 + T * 16),
        # + block 0's input LayerNorm: its output row and (mean, rstd) written; the backward reads the LN output's
        # gradient and the statistics too (the unfused LayerNorm pass re-read the embedding output instead)
        "asme_embedding_ln_fwd": ("hbm", T * 8 + 3 * T * d * 4 + T * 16 + T * 8),
        "asme_embedding_ln_bwd": ("hbm", T * 8 + 4 * T * d * 4 + T * 16 + T * 8),
        "asme_lazy_adam_apply": ("hbm", U * 8 + U * d * 4 + 6 * U * d * 4 + U * 4),
        "asme_lazy_adam_catch_up": ("hbm", U * 8 + 6 * U * d * 4 + 2 * U * 4),
        # staged form: the same rows read (random) and written to the compact staging rows (slot order); the apply
        # reads those + the compact gradient (slot order) and writes the table rows (random) + last_step
        "asme_lazy_adam_stage": ("hbm", U * 8 + U * 4 + 6 * U * d * 4),
        "asme_lazy_adam_apply_staged": ("hbm", U * 8 + U * d * 4 + 6 * U * d * 4 + U * 4),
        # sampled head: h read once, the distinct pos / neg rows gathered (U_pn), two logits written (fwd); the bwd
        # reads the ids, the rows and the two logit gradients and writes dh -- h only where it also scatters the
        # table gradient (table_grad="dense"; the sparse plan takes the table's rows from the step's contributions)
        "asme_sampled_logits_fwd": ("hbm", T * d * 4 + 2 * T * 8 + U_pn * d * 4 + 2 * T * 4),
        "asme_sampled_logits_bwd": ("hbm", 2 * T * 8 + U_pn * d * 4 + 2 * T * 4 + T * d * 4
                                    + (T * d * 4 if args.table_grad == "dense" else 0)),
        "asme_gelu_dropout_bwd": ("hbm", 3 * T * ffn * 4),
        "asme_adam_rows_step": ("hbm", 6 * V * d * 4 + V * 4 + U * d * 4),
        # session items read once + x / pos / neg written (the in-session membership scans hit the cache)
        "asme_posneg_sample": ("hbm", B * (L + 1) * 8 + 3 * B * L * 8 + B * 8),
        # the step's n = 3T table ids: read once, the slot map probed per id and written per unique row, the
        # inverse (n) and the unique ids (U) written
        "asme_dedup_ids": ("hbm", 3 * T * (8 + 4 + 8) + U * (8 + 4)),
        # (the training step's form: the three id tensors read in place as segments, same bytes)
        "asme_dedup_ids_segments": ("hbm", 3 * T * (8 + 4 + 8) + U * (8 + 4)),
        # occurrence CSR: the inverse read, order + sorted slot written (int32), the U + 1 segment offsets
        "asme_occurrence_csr": ("hbm", 3 * T * (8 + 4 + 4) + 4 * (U + 1)),
        # ordered per-row sums + the lazy Adam step: the three contributions' rows (embedding d_rows, h for the
        # pos and for the neg ids) + their scales, order / slot per occurrence, the staged p / m / v read, the
        # table's p / m / v rows + last_step written, the unique ids read
        # position-embedding gradient: d_rows read once, 32 chunk partials (L, d) written and read, (L, d) written
        "asme_position_grad": ("hbm", T * d * 4 + 2 * 32 * L * d * 4 + L * d * 4),
        # LayerNorm parameter partials summed (mean over the step's launches: the four residual-LN backwards' 1,024 x
        # 2d and the embedding backward's 2,048 x 6d)
        "asme_reduce_rows": ("hbm", (4 * 1024 * 2 * d + 2048 * 6 * d) * 4 / 5),
        # the sampled BCE loss: two logits + the mask read (fwd), + two logit gradients written (bwd)
        "asme_sasrec_bce_fwd": ("hbm", 2 * T * 4 + T),
        "asme_sasrec_bce_bwd": ("hbm", 4 * T * 4 + T),
        "asme_table_grad_reduce_apply": ("hbm", 3 * T * d * 4 + 2 * T * 4 + 3 * T * 8 + 6 * U * d * 4 + U * 12),
    }
    # HBM traffic per launch from the committed rocprofv3 PMC pass (FETCH_SIZE x2 + WRITE_SIZE, gfx950
    # corrections of MI355X_MICROARCH.md §HBM; tools/pmc_traffic.py) for this exact configuration
    traffic = {}
    tp = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tp):
        with open(tp) as f:
            tj = json.load(f)
        if tj.get("config") == {"batch": B, "seq_len": L, "items": args.items, "dim": d, "layers": args.layers}:
            traffic = dict(tj.get("bytes_per_launch", {}))
            if "asme_dedup_ids" in traffic:  # tools/pmc_traffic.py attributes the segmented dedup's kernels to it
                traffic.setdefault("asme_dedup_ids_segments", traffic["asme_dedup_ids"])
    mb = committed_profile("mfma_busy.json", {"batch": B, "seq_len": L, "items": args.items, "dim": d,
                                              "layers": args.layers})
    rooflines = roofline_entries(kstats, work, traffic, mb.get("mfma_busy"))
    roof = rooflines[0] if rooflines else None

    result = {
        "metric": ("training sequences/sec at B=1024 L=200 |I|=10M (SASRec-neg, fwd+bwd+Adam)" if ids_kind == "uniform"
                   else f"training sequences/sec (SASRec-neg, {ids_kind} ids, B={B} L={L} |I|={args.items}, fwd+bwd+Adam)"),
        "value": round(value, 2), "unit": "sequences/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "fp32", "data": (f"synthetic sessions ({ids_kind} ids), a fresh GPU-sampled batch every step, random-init weights"
                                                 if args.producer == "gpu" else
                                                 f"synthetic ({ids_kind} ids, two resident batches), random-init weights"),
        "config": {"workload": "sasrec-neg train step", "model": "SASRec", "global_batch": B * world,
                   "batch_per_gpu": B, "seq_len": L, "items": args.items, "dim": d, "heads": args.heads,
                   "layers": args.layers, "dropout": args.dropout, "table_grad": args.table_grad,
                   "ids": ids_kind, "producer": args.producer,
                   "ids_ahead": (args.ids_ahead if args.producer == "gpu" and not sharded else "off"),
                   "overlap_negatives": bool(overlap and sharded and world > 1),
                   "parallelism": f"dp{world}+rowshard{world}" if sharded else "single"},
        "roofline": roof,
        "rooflines": rooflines,
        "flush_ms": round(flush_ms, 3),
        # diagnostic: median host time to issue one step's launches (the GPU runs behind the host when it is smaller)
        "host_issue_ms": round(1000 * sorted(host_s)[len(host_s) // 2], 3),
        "ids_ahead_hits": getattr(module, "ids_ahead_hits", 0),
        "cpu_baseline": None,
    }
    if eval_leg is not None:
        result["eval"] = eval_leg
    del model, module, opt, batches
    torch.cuda.empty_cache()
    return result


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def resolve_world(args, env=None):
    """(world, must_launch): the rank count this invocation runs as.  `--gpus N` with no WORLD_SIZE in the
    environment and N > 1 means "launch N ranks myself" (launch_ranks); under a launcher (torchrun sets WORLD_SIZE)
    the launcher's world size must equal --gpus, so the printed n_gpus can never disagree with the flag."""
    env = os.environ if env is None else env
    if args.gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return args.gpus, args.gpus > 1
    if int(ws) != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {args.gpus}: they must agree")
    return int(ws), False


def rank_envs(n, port, base=None):
    """the environment of each spawned rank (one process per GPU, torch.distributed's env:// rendezvous on
    127.0.0.1; HSA_ENABLE_IPC_MODE_LEGACY and the rest of the parent's environment are inherited)"""
    base = dict(os.environ if base is None else base)
    out = []
    for r in range(n):
        e = dict(base)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        out.append(e)
    return out


def launch_ranks(args, argv=None, script=None) -> int:
    """`python bench.py --gpus N` without a launcher: start N rank processes of this same script (one per GPU) and
    wait for them.  This parent never touches the GPU (torch.cuda.device_count() does not initialise HIP on this
    image), so no process that owns a GPU context is forked or exec'ed.  If any rank fails the others are
    terminated (exactly the PIDs started here) and its exit code is returned; rank 0 prints the one JSON line."""
    import signal
    import subprocess
    n = args.gpus
    if args.backend == "nccl":
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} GPUs, {have} visible (use --backend gloo to rehearse several "
                  f"ranks on fewer GPUs)", file=sys.stderr, flush=True)
            return 2
    argv = sys.argv[1:] if argv is None else argv
    script = os.path.abspath(__file__) if script is None else script
    procs = [subprocess.Popen([sys.executable, "-u", script] + list(argv), env=e)
             for e in rank_envs(n, free_port())]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc:
        print(f"bench.py: a rank exited with status {rc}; the remaining ranks were stopped", file=sys.stderr,
              flush=True)
    return rc


def main():
    args = parse()
    world, must_launch = resolve_world(args)
    if must_launch:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.backend == "gloo":
        local = local % torch.cuda.device_count()  # rehearsal: several ranks may share one GPU
    if world > 1 or args.sharded:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    if args.main_stream == "high":
        torch.cuda.set_stream(torch.cuda.Stream(dev, priority=-1))
    asme = __graft_entry__.load_package()
    V = args.items + 3
    B, L, d = args.batch, args.seq_len, args.dim

    torch.manual_seed(rank)
    if args.workload in ("bert4rec", "kebert4rec"):
        result = bench_bert4rec(args, asme, dev, world, rank, args.workload, args.items)
        if rank == 0:
            emit(result, args)
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    result = bench_sasrec(args, asme, dev, world, rank, args.ids)
    # the other BASELINE workloads, measured in the same run (same contract: warm-up, barrier + synchronize around
    # exactly --steps steps, max over ranks) and reported inside this one JSON line
    legs = parse_legs(args.legs)
    if legs:
        result["workloads"] = {}
        for leg, items in legs:
            torch.manual_seed(rank)
            if leg == "sasrec_zipf":
                if args.ids == "zipf":
                    continue  # the headline already is the Zipf run
                result["workloads"][leg] = bench_sasrec(args, asme, dev, world, rank, "zipf", with_eval=False)
            elif leg == "sasrec_overlap":
                # the headline step with the negative-only rows in a second, overlapped exchange (sharded.py
                # overlap_negatives): where rows cross the fabric (N > 1), or on a 1-rank RCCL group with --sharded
                if world == 1 and not args.sharded:
                    continue
                result["workloads"][leg] = bench_sasrec(args, asme, dev, world, rank, args.ids, with_eval=False,
                                                        overlap=True)
            else:
                result["workloads"][leg] = bench_bert4rec(args, asme, dev, world, rank, leg, items)
            torch.cuda.empty_cache()
    if rank == 0 and world == 1 and args.cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, V)
    if rank == 0:
        emit(result, args)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
