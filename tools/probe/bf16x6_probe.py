"""Error of bf16-split fp32 GEMM tiles vs float64, against the native fp32 MFMA (see bf16x6_probe.hip).
Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/probe/bf16x6_probe.hip -o tools/probe/libbf16x6.so"""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbf16x6.so"))
lib.run_probe.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p]
names = {0: "fp32 mfma", 1: "bf16x6 1acc", 2: "bf16x6 2acc", 3: "bf16x3"}
torch.manual_seed(0)
for K in (128, 512):
    for dist in ("normal", "uniform+", "wide"):
        T = 2048
        if dist == "normal":
            A = torch.randn(T * 16, K, dtype=torch.float64)
            B = torch.randn(T * 16, K, dtype=torch.float64)
        elif dist == "uniform+":
            A = torch.rand(T * 16, K, dtype=torch.float64)
            B = torch.rand(T * 16, K, dtype=torch.float64)
        else:
            A = torch.randn(T * 16, K, dtype=torch.float64) * torch.exp(torch.randn(T * 16, K, dtype=torch.float64) * 3)
            B = torch.randn(T * 16, K, dtype=torch.float64) * torch.exp(torch.randn(T * 16, K, dtype=torch.float64) * 3)
        A32, B32 = A.float(), B.float()
        ref = torch.einsum("tik,tjk->tij", A32.double().view(T, 16, K), B32.double().view(T, 16, K))
        scale = torch.einsum("tik,tjk->tij", A32.double().abs().view(T, 16, K), B32.double().abs().view(T, 16, K))
        Ad, Bd = A32.cuda(), B32.cuda()
        line = []
        for mode in (0, 1, 2, 3):
            C = torch.empty(T * 16, 16, device="cuda")
            lib.run_probe(Ad.data_ptr(), Bd.data_ptr(), C.data_ptr(), T, K, mode, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            err = (C.cpu().double().view(T, 16, 16) - ref).abs() / scale
            line.append(f"{names[mode]}: max {err.max().item():.2e} mean {err.mean().item():.2e}")
        print(f"K={K} {dist:8s} | " + " | ".join(line))
