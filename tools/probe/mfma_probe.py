import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("PROBE_LIB", "libprobe.so")))
lib.run_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.empty(4096 * 256, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for nacc in (4, 8, 16):
    for blocks in (256, 512, 1024, 2048):
        iters = 2000
        lib.run_probe(nacc, blocks, iters, out.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); lib.run_probe(nacc, blocks, iters, out.data_ptr(), s); e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        flops = blocks * 4 * iters * nacc * 2048.0
        print(f"nacc={nacc} blocks={blocks}: {flops / ms / 1e9:.1f} TF/s")
