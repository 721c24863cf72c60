"""CPU-side checks of the drop-in boundary: libdsgan_hip.so loads, exports every symbol that
include/dsgan_hip.h declares with the argument counts the ctypes table uses; no compute call."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dsgan_hip.h")


def _header_decls():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(?:int|long|const char\*)\s+(dsgan_\w+)\s*\(([^)]*)\)\s*;", txt):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        decls[m.group(1)] = len(args)
    return decls


def _lib_or_skip():
    from dsgan_hip import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libdsgan_hip.so not built (run __graft_entry__.build())")
    return _lib


def test_header_matches_ctypes_table():
    from dsgan_hip._lib import SIGNATURES
    decls = _header_decls()
    assert set(decls) == set(SIGNATURES), set(decls) ^ set(SIGNATURES)
    for name, n in decls.items():
        assert len(SIGNATURES[name]) == n, (name, n, len(SIGNATURES[name]))


def test_library_exports_every_symbol():
    _lib = _lib_or_skip()
    lib = _lib.load()
    for name in _header_decls():
        assert hasattr(lib, name), name
    assert lib.dsgan_abi_version() == 3
    assert lib.dsgan_last_error_string() is not None


def test_every_scratch_argument_carries_its_size():
    """The scratch contract of include/dsgan_hip.h: a `float* ws` / `float* work` parameter is always
    followed by its element count, and the ctypes table passes a long there."""
    from dsgan_hip._lib import SIGNATURES, L
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    seen = 0
    for m in re.finditer(r"\b(?:int|long|const char\*)\s+(dsgan_\w+)\s*\(([^)]*)\)\s*;", txt):
        args = [" ".join(a.split()) for a in m.group(2).split(",")]
        for i, a in enumerate(args):
            if a in ("float* ws", "float* work"):
                seen += 1
                nxt = args[i + 1] if i + 1 < len(args) else ""
                assert nxt in ("long ws_elems", "long work_elems"), (m.group(1), a, nxt)
                assert SIGNATURES[m.group(1)][i + 1] is L, m.group(1)
    assert seen >= 20


def test_bad_args_fail_loudly_without_gpu_work():
    """Argument validation runs on the host before any launch."""
    _lib = _lib_or_skip()
    with pytest.raises(RuntimeError, match="bad geometry"):
        _lib.call("dsgan_conv_fwd", None, 0, None, None, None, 0, None, 0, 0, 3, 8, 8, 4, 1, 1, 1, 0,
                  8, 8, 0, 0.2, 0, 0, 0, None)
    with pytest.raises(RuntimeError, match="K must be odd"):
        _lib.call("dsgan_dwconv_fwd", 1, 0, 1, None, 1, 0, 1, 1, 8, 8, 4, 0, 0, None)


def test_ptr_refuses_cpu_tensors():
    import torch
    from dsgan_hip._lib import ptr
    with pytest.raises(RuntimeError, match="device tensor"):
        ptr(torch.zeros(3))


def test_model_refuses_cpu_device():
    from options.train_options import default_train_opt
    from models import create_model
    opt = default_train_opt(gpu_ids=[])
    with pytest.raises(RuntimeError, match="needs a ROCm GPU"):
        create_model(opt)
