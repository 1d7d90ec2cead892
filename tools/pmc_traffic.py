"""HBM traffic per C-ABI call from a rocprofv3 FETCH_SIZE / WRITE_SIZE pass over bench.py.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes of 16-B/lane streaming
reads -> x2; WRITE_SIZE is exact for 16-B stores; both are reported in KiB.  An API call that launches
several kernels is the sum of its kernels; the per-call value is the median over calls (the end-of-run
flush launch of the lazy-Adam catch-up is an outlier, not a step).
Usage: python tools/pmc_traffic.py <dir with pmc_FETCH_SIZE/ pmc_WRITE_SIZE/> <out.json> B L ITEMS DIM LAYERS [WORKLOAD]
"""
import collections
import csv
import json
import re
import statistics
import sys

# kernel-name regex -> (API call, counts-the-call?)
MAP = [
    (r"attn_fwd(_res)?_kernel", "asme_attention_fwd", True),
    # the backward: dK/dV (storing dS) first, then dQ = dS K (resident path); the streaming path's dQ pass first
    (r"attn_bwd_dkdv_res_kernel<\d+, true>", "asme_attention_bwd", True),
    (r"attn_bwd_dq_ds_kernel", "asme_attention_bwd", False),
    (r"attn_bwd_dq(_res)?_kernel", "asme_attention_bwd", True),
    (r"attn_bwd_dkdv(_res)?_kernel", "asme_attention_bwd", False),
    (r"weight_grad_kernel", "asme_linear_weight_grad", True),
    (r"sum_slabs(_cols)?_kernel", "asme_linear_weight_grad", False),
    # <RowLayout, k, LN3, LN2>: LN3 (block 0's input LayerNorm fused) makes the call the _ln form
    (r"emb_fwd4_kernel<asme::RowLayout<[^>]*>, \d+, true", "asme_embedding_ln_fwd", True),
    (r"emb_bwd4_kernel<asme::RowLayout<[^>]*>, \d+, true", "asme_embedding_ln_bwd", True),
    (r"emb_bwd128_kernel<true", "asme_embedding_ln_bwd", True),  # (LN3: the fused next LayerNorm)
    (r"emb_bwd128_kernel", "asme_embedding_bwd", True),
    (r"emb_fwd4?_kernel", "asme_embedding_fwd", True),
    (r"emb_bwd4?_kernel", "asme_embedding_bwd", True),
    (r"lazy_catch_up(_v4)?_kernel", "asme_lazy_adam_catch_up", True),
    (r"lazy_apply(_v4)?_kernel", "asme_lazy_adam_apply", True),
    (r"lazy_stage_v4_kernel", "asme_lazy_adam_stage", True),
    (r"lazy_row_kernel<\d+, true>", "asme_lazy_adam_stage", True),
    (r"lazy_pipe_kernel<\d+, \d+, \d+, true>", "asme_lazy_adam_stage", True),
    (r"lazy_apply_staged_v4_kernel", "asme_lazy_adam_apply_staged", True),
    (r"sampled_fwd4?_kernel", "asme_sampled_logits_fwd", True),
    (r"sampled_bwd4?_kernel", "asme_sampled_logits_bwd", True),
    (r"posneg_kernel", "asme_posneg_sample", True),
    # the sparse table gradient: dedup (claim .. inverse), occurrence CSR (csr_*), ordered sums + Adam (grad_*)
    (r"claim_kernel", "asme_dedup_ids", True),
    (r"(flag|compact|inverse|dedup_\w+)_kernel", "asme_dedup_ids", False),
    (r"csr_count_kernel", "asme_occurrence_csr", True),
    (r"(csr_\w+|chained_scan)_kernel", "asme_occurrence_csr", False),
    (r"grad_chunk_kernel<true>", "asme_table_grad_reduce_apply", True),
    (r"grad_span_kernel<true>", "asme_table_grad_reduce_apply", False),
    (r"gelu_dropout_fwd_kernel", "asme_gelu_dropout_fwd", True),
    (r"gelu_dropout_bwd_kernel", "asme_gelu_dropout_bwd", True),
    (r"residual_ln_fwd_kernel", "asme_residual_ln_fwd", True),
    (r"residual_ln_bwd_kernel", "asme_residual_ln_bwd", True),
    (r"ws_gemm_kernel", "asme_ws_linear", True),
    (r"pos_partial_kernel", "asme_position_grad", True),
    (r"reduce_rows_kernel", "asme_reduce_rows", True),
    (r"bce_fwd_kernel", "asme_sasrec_bce_fwd", True),
    (r"bce_finish_kernel", "asme_sasrec_bce_fwd", False),
    (r"bce_bwd_kernel", "asme_sasrec_bce_bwd", True),
    # the fused logits + CE head (csrc/logits.hip): the engine's mode names the call; the operand splits that open
    # a call are attributed to the call of the engine launch that follows them (see per_call)
    # (api None: the kernel belongs to the logits call that launched the previous mapped kernel)
    # (the gradient passes run on logits_grad16_kernel / logits_grad_kernel: same mode numbers)
    (r"logits_engine_kernel<0", "asme_linear_xent_fwd", True),
    (r"logits_(engine|grad16|grad)_kernel<4", "asme_linear_xent_fwd_dh", True),
    (r"logits_(engine|grad16|grad)_kernel<1", "asme_linear_xent_bwd", True),
    (r"scale_rows_kernel", "asme_linear_xent_bwd_dw", True),
    (r"logits_(engine|grad16|grad)_kernel<2", None, False),
    (r"(lce_rows|lce_finish|fdh_finish|sum_parts)_kernel", None, False),
]
PENDING = r"split_planes_kernel"  # belongs to the next mapped logits kernel's call
# calls whose launches have different shapes (the bench's work figure is their mean): mean, not median
MEAN = {"asme_ws_linear", "asme_linear_weight_grad", "asme_reduce_rows"}


def load(path, counter):
    out = []  # (dispatch id, kernel, bytes)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    return sorted(out)


def per_call(rows, scale):
    calls = collections.defaultdict(list)
    cur = {}
    pending = 0.0
    last = None
    for _, name, b in rows:
        if re.search(PENDING, name):
            pending += b * scale
            continue
        for rx, api, counts in MAP:
            if re.search(rx, name):
                if api is None:
                    if last is None:
                        break
                    api = last
                if counts or api not in cur:
                    calls[api].append(0.0)
                    cur[api] = True
                calls[api][-1] += b * scale + pending
                pending = 0.0
                last = api
                break
    return calls


def main():
    d, out = sys.argv[1], sys.argv[2]
    B, L, items, dim, layers = (int(x) for x in sys.argv[3:8])
    f = per_call(load(f"{d}/pmc_FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE"), 2.0)
    w = per_call(load(f"{d}/pmc_WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE"), 1.0)
    res = {}
    for api in sorted(set(f) | set(w)):
        n = min(len(f.get(api, [])), len(w.get(api, [])))
        if n == 0:
            continue
        tot = [f[api][i] + w[api][i] for i in range(n)]
        res[api] = round(statistics.mean(tot) if api in MEAN else statistics.median(tot))
    wl = sys.argv[8] if len(sys.argv) > 8 else "sasrec-neg"
    json.dump({"config": {"batch": B, "seq_len": L, "items": items, "dim": dim, "layers": layers},
               "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over bench.py --workload {wl} "
                         "--steps 2",
               "bytes_per_launch": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
