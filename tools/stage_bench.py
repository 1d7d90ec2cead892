"""asme_lazy_adam_stage / _apply_staged on U = 590k random unique rows of a (V, 128) table: the memory side (no
replay: every row already current) and with a fixed replay length, for two table sizes (page / TLB reach).
Usage: python tools/stage_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402


def timed(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    asme = __graft_entry__.load_package()
    call, ptr, st = asme._lib.call, asme._lib.ptr, asme._lib.stream
    dev = torch.device("cuda", 0)
    D, U, upto = 128, 590_000, 25
    for V in (1_000_000, 10_000_000):
        p = torch.randn(V, D, device=dev) * 0.01
        m = torch.zeros(V, D, device=dev)
        v = torch.zeros(V, D, device=dev)
        hist = torch.zeros(1024, 8, device=dev)
        for t in range(1, upto + 1):
            call("asme_lazy_adam_record_step", ptr(hist), hist.shape[0], t, 1e-3, 0.99, 0.998, 1e-8, 1e-3, st())
        rows = torch.randperm(V, device=dev)[:U].contiguous()
        count = torch.tensor([U], dtype=torch.int32, device=dev)
        staged = torch.empty(3, U, D, device=dev)
        grad = torch.randn(U, D, device=dev)
        for back in (0, 12):
            last = torch.full((V,), upto - back, dtype=torch.int32, device=dev)
            f = lambda: call("asme_lazy_adam_stage", ptr(rows), ptr(count), U, ptr(last), ptr(p), ptr(m), ptr(v), D,  # noqa
                             ptr(hist), hist.shape[0], upto, ptr(staged[0]), ptr(staged[1]), ptr(staged[2]), st())
            t = timed(f)
            print(f"V={V:>9} replay={back:2d}: stage {t:6.1f} us  {U * (6 * D * 4 + 12) / t / 1e3:5.0f} GB/s")
        last.fill_(upto)
        a = lambda: call("asme_lazy_adam_apply_staged", ptr(rows), ptr(count), U, ptr(grad), ptr(staged[0]),  # noqa
                         ptr(staged[1]), ptr(staged[2]), ptr(last), ptr(p), ptr(m), ptr(v), D, ptr(hist),
                         hist.shape[0], upto, st())
        t = timed(a)
        print(f"V={V:>9}: apply_staged {t:6.1f} us  {U * (7 * D * 4 + 12) / t / 1e3:5.0f} GB/s")
        del p, m, v, staged, grad


if __name__ == "__main__":
    main()
