"""CPU: the host side of the C-ABI under AddressSanitizer ("-fsanitize=address host build of the C-ABI
shim").  `make asan` builds every source with -fsanitize=address on the host code only (csrc/Makefile); the driver
(tests/native/asan_drive.py) loads that library with the ASan runtime preloaded and NO GPU visible, and calls every
entry point of include/asme_mi.h: the size / support queries over a sweep of sizes (0, negative, 2^31, 2^40 ...),
every compute entry point with null pointers and sizes 1, 0 and -1 (each must be rejected with status -1 and a
message) and with host stand-in pointers (validation passes, the launch fails with status -2 and a message: no
device).  A crash, an ASan report or a silent acceptance fails the test.  (It found the division by zero of
asme_linear_weight_grad_workspace for zero-sized shapes, fixed in csrc/gemm.hip.)"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "recsys-22-user-attributes-recommender_amd", "csrc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.timeout(900)
def test_c_abi_host_code_under_asan():
    if not os.path.exists(CLANG):
        pytest.skip("no ROCm toolchain")
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-C", CSRC, "asan", f"-j{jobs}"], check=True, stdout=subprocess.DEVNULL)
    rt = subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"], check=True, capture_output=True,
                        text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    r = subprocess.run(["python3", os.path.join(ROOT, "tests", "native", "asan_drive.py"),
                        os.path.join(CSRC, "build", "asan", "libasme_mi_asan.so")],
                       env=env, capture_output=True, text=True, timeout=300)
    assert "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads(r.stdout.strip().splitlines()[0])
    assert out["bad"] == []
    c = out["counts"]
    assert out["functions"] >= 90 and c["queries"] > 0
    assert c["rejected"] >= 3 * (out["functions"] - 25)  # null pointers / sizes 0 and -1: rejected by validation
