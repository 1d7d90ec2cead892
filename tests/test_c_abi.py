"""CPU: the C-ABI shared library loads and exports every entry point include/asme_mi.h declares;
argument validation fails loudly (status -1 + message) without touching a GPU."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "asme_mi.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(asme_\w+)\s*\(", text))


def test_header_and_binding_agree(asme):
    assert _declared() == set(asme._lib.SIGNATURES)


def test_library_exports_every_declared_symbol(asme):
    lib = asme._lib.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.asme_mi_abi_version() == 1


def test_argument_validation_is_loud(asme):
    lib = asme._lib.load()
    rc = lib.asme_embedding_fwd(None, 4, 2, None, 10, 8, None, None, None, 1e-5, 0.0, 0, None, None, None, 1e-5,
                                0.0, 0, None, None, None, None, None)
    assert rc == -1
    assert b"null pointer" in lib.asme_mi_last_error()
    with pytest.raises(asme._lib.ASMEKernelError):
        asme._lib.call("asme_attention_fwd", 8, 8, 8, 0, 0, 0, None, 1, 1, 2000, 64, 1, 1.0, 0.0, 0, 8, 0, 8, None, None)


def test_dedup_workspace_query_is_host_only(asme):
    lib = asme._lib.load()
    assert lib.asme_dedup_workspace_bytes(1 << 20) >= 4 * (1 << 20)


def test_cpu_tensors_are_rejected(asme):
    import torch
    with pytest.raises(asme._lib.ASMEKernelError, match="no CPU fallback"):
        asme.ops.gelu_dropout(torch.randn(8), 0.0)
