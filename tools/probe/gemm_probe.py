import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgemm.so"))
lib.run_gemm_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
s = torch.cuda.current_stream().cuda_stream
T = 204800
for K, N in [(128, 128), (128, 512), (512, 128)]:
    x = torch.randn(T, K, device="cuda"); w = torch.randn(N, K, device="cuda"); y = torch.empty(T, N, device="cuda")
    for grid in (512, 1024):
        res = []
        for mode in range(4):
            f = lambda: lib.run_gemm_probe(mode, x.data_ptr(), T, K, w.data_ptr(), N, y.data_ptr(), grid, s)
            for _ in range(3): f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10): f()
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            res.append(f"{2.0*T*K*N/ms/1e9:6.1f}")
        print(f"K={K} N={N} grid={grid}: full/noepi/noload/neither TF/s = {' '.join(res)}")
