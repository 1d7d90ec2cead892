"""Lazy-Adam full flush at the bench table size (10M x 128): time + effective bandwidth.
Usage: python tools/flush_bench.py [--rows N] [--k STEPS]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=13)
    ap.add_argument("--wd", type=float, default=0.0)
    ap.add_argument("--spread", action="store_true",
                    help="each row's last step drawn geometric(p = 0.059) back from k (uniform ids at 590k of 10M rows "
                         "per step), instead of every row at step 0")
    a = ap.parse_args()
    asme = __graft_entry__.load_package()
    call, ptr, st = asme._lib.call, asme._lib.ptr, asme._lib.stream
    dev = torch.device("cuda", 0)
    V, D = a.rows, 128
    p = torch.randn(V, D, device=dev) * 0.01
    m = torch.zeros(V, D, device=dev)
    v = torch.zeros(V, D, device=dev)
    hist = torch.zeros(1024, 8, device=dev)
    for t in range(1, a.k + 1):
        call("asme_lazy_adam_record_step", ptr(hist), hist.shape[0], t, 1e-3, 0.9, 0.999, 1e-8, a.wd, st())
    last = torch.zeros(V, dtype=torch.int32, device=dev)
    times = []
    if a.spread:
        g = torch.Generator(device=dev).manual_seed(1)
        u = torch.rand(V, device=dev, generator=g)
        back = torch.floor(torch.log1p(-u) / torch.log1p(torch.tensor(-0.059, device=dev))).clamp(max=a.k)
        last_init = (a.k - back).to(torch.int32)
    else:
        last_init = torch.zeros(V, dtype=torch.int32, device=dev)
    for rep in range(4):
        last.copy_(last_init)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("asme_lazy_adam_catch_up", None, None, V, ptr(last), ptr(p), ptr(m), ptr(v), D, ptr(hist), hist.shape[0], a.k, st())
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    t = min(times[1:])
    gb = V * D * 4 * 6 / 1e9
    print(f"flush {V} x {D}, k={a.k} wd={a.wd} spread={a.spread}: {t:.2f} ms  {gb / t:.2f} TB/s (algorithmic {gb:.1f} GB)")


if __name__ == "__main__":
    main()
