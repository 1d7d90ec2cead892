import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("PROBE_LIB", "libprobe2.so")))
lib.run_probe2.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.empty(4096 * 256, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for nacc in (8, 16):
    for mode in range(4):
        for blocks in (256, 512):
            iters = 500
            lib.run_probe2(nacc, mode, blocks, iters, out.data_ptr(), s)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); lib.run_probe2(nacc, mode, blocks, iters, out.data_ptr(), s); e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            flops = blocks * 4 * iters * 4 * nacc * 2048.0
            print(f"nacc={nacc} mode={mode} blocks={blocks}: {flops / ms / 1e9:.1f} TF/s")
