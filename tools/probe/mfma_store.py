import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libms.so"))
lib.run_ms.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
out = torch.empty(1024 * 4 * 100 * 2048 + (1 << 22), device="cuda")
s = torch.cuda.current_stream().cuda_stream
for mode in (4, 1, 5, 6):
    for blocks in (512, 1024):
        tiles = 100 if mode != 6 else 25
        waves = blocks * 4
        need = tiles * waves * 2048 if mode == 5 else (tiles * waves // 4) * 16 * 512 if mode == 6 else 0
        assert need <= out.numel(), (mode, need, out.numel())
        lib.run_ms(mode, blocks, tiles, out.data_ptr(), s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); lib.run_ms(mode, blocks, tiles, out.data_ptr(), s); e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        flops = blocks * 4 * tiles * 256 * 2048.0
        print(f"mode={mode} blocks={blocks}: {flops / ms / 1e9:.1f} TF/s  ({ms * 1e3:.0f} us)")
