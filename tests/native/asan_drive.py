"""Drive every C-ABI entry point of the host-ASan build (csrc/Makefile `asan`) through its host code without a GPU.

Run by tests/test_asan_host.py in a subprocess with the ASan runtime preloaded and no GPU visible.  torch is NOT
imported (the binding table is read from _lib.py's source), so the only instrumented code is the library's own host
code: argument validation, workspace / support queries, launch configuration.  Every call must return a status
(0 = accepted, -1 = rejected with a message, -2 = HIP error with a message: no device here) -- a crash or an ASan
report fails the test.  Prints one summary line of JSON."""
import ast
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(os.path.dirname(HERE)), "recsys-22-user-attributes-recommender_amd")
lib = ctypes.CDLL(sys.argv[1])

src = open(os.path.join(PKG, "_lib.py")).read()
tree = ast.parse(src)
sigs = restypes = None
for node in tree.body:
    if isinstance(node, ast.AnnAssign) and getattr(node.target, "id", "") == "SIGNATURES":
        sigs = node.value
    if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", "") == "SIGNATURES":
        sigs = node.value
    if isinstance(node, ast.Assign) and getattr(node.targets[0], "id", "") == "_RESTYPES":
        restypes = node.value
names = {"p": ctypes.c_void_p, "i64": ctypes.c_int64, "i32": ctypes.c_int, "f32": ctypes.c_float,
         "u64": ctypes.c_uint64, "f64": ctypes.c_double, "ctypes": ctypes}
SIG = eval(compile(ast.Expression(sigs), "sig", "eval"), names)
RES = eval(compile(ast.Expression(restypes), "res", "eval"), names)

for name, args in SIG.items():
    fn = getattr(lib, name)
    fn.argtypes = args
    fn.restype = RES.get(name, ctypes.c_int)
lib.asme_mi_last_error.restype = ctypes.c_char_p

queries = {n for n, r in RES.items() if r is ctypes.c_int64} | {n for n in SIG if n.endswith("_supported")} | {
    "asme_embedding_bwd_partials_count", "asme_mi_abi_version"}
counts = {"rejected": 0, "hip_error": 0, "accepted": 0, "queries": 0}
bad = []
hip_errors = []


def arg(t, size, ptr):
    if t is ctypes.c_void_p:
        return ptr
    if t in (ctypes.c_float, ctypes.c_double):
        return 0.5
    return size


# a host buffer standing in for a device pointer: no call may dereference a device pointer on the host, and the
# HIP launch it would reach fails without a device
buf = ctypes.create_string_buffer(1 << 16)
for name, args in SIG.items():
    fn = getattr(lib, name)
    if name == "asme_mi_last_error":
        continue
    if name in queries:  # host-only size / support queries over a sweep, including absurd sizes
        for v in (0, 1, 2, 3, 31, 64, 100, 128, 200, 384, 512, 4096, 65537, 10_000_003, 1 << 31, 1 << 40, -1):
            fn(*[arg(t, v, None) for t in args])
            counts["queries"] += 1
        continue
    for size, ptr in ((1, None), (0, None), (-1, None), (7, ctypes.addressof(buf))):
        # (the host array arguments of asme_adam_step: real host arrays of "device" pointers)
        if name == "asme_adam_step" and ptr is not None:
            arr = (ctypes.c_void_p * 7)(*([ctypes.addressof(buf)] * 7))
            nn = (ctypes.c_int64 * 7)(*([7] * 7))
            call_args = [7, arr, arr, arr, arr, nn] + [0.5] * 5 + [1, None]
        else:
            call_args = [arg(t, size, ptr) for t in args]
        rc = fn(*call_args)
        msg = lib.asme_mi_last_error() or b""
        if rc == -1:
            counts["rejected"] += 1
        elif rc == -2:
            counts["hip_error"] += 1
            hip_errors.append((name, size, ptr is not None))
        elif rc == 0:
            counts["accepted"] += 1
        else:
            bad.append((name, size, rc))
        if rc in (-1, -2) and not msg:
            bad.append((name, size, "no message"))
        if size == 1 and ptr is None and rc == 0:
            bad.append((name, size, "null pointers accepted"))
print(json.dumps({"functions": len(SIG), "counts": counts, "bad": bad}))
if os.environ.get("ASAN_DRIVE_VERBOSE"):
    print(hip_errors)
sys.exit(1 if bad else 0)
