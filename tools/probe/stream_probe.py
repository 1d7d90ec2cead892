"""Achievable HBM rates of the embedding kernels' patterns (tools/probe/stream_probe.hip), T = 204,800 rows of 512 B:
1 read -> 2 writes (forward), 4 reads -> 1 write (backward), read-only, write-only; cached vs non-temporal stores;
one-shot grid vs grid-stride.  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC stream_probe.hip -o libstream.so"""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libstream.so"))
lib.run_stream.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 6 + [ctypes.c_int64, ctypes.c_void_p]
T, D = 204800, 128
n = T * D // 4
bufs = [torch.randn(T, D, device="cuda") for _ in range(6)]
s = torch.cuda.current_stream().cuda_stream
nbytes = {0: 3, 1: 5, 2: 1, 3: 1}
for mode in (0, 1, 2, 3):
    for nt in (0, 1):
        for blocks in (n // 256, 2048, 4096, 8192):
            args = [mode, nt, blocks] + [b.data_ptr() for b in bufs] + [n, s]
            for _ in range(3):
                lib.run_stream(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                lib.run_stream(*args)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            gb = nbytes[mode] * T * D * 4
            print(f"mode={mode} nt={nt} blocks={blocks}: {us:.1f} us  {gb / us / 1e3:.0f} GB/s ({gb / us / 8e6:.3f})",
                  flush=True)
