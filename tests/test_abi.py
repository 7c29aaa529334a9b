"""CPU-side checks of the drop-in boundary: the in-tree C-ABI library loads and
exports every symbol include/bann.h declares; the Python binding covers them
all; no compute is called (no GPU here)."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(glob.glob(os.path.join(ROOT, "include", "*.h")))
LIB = os.path.join(ROOT, "rs-bann_amd", "librsbann_amd.so")


def header_functions():
    """every function declared in include/*.h (bann.h, bann_net.h)"""
    fns = set()
    for h in HEADERS:
        txt = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        fns |= set(re.findall(r"\b(bann_[a-z_0-9]+)\s*\(", txt))
    return sorted(fns)


def test_header_parses():
    fns = header_functions()
    assert len(HEADERS) >= 2
    assert "bann_ctx_create" in fns and "bann_hmc_step" in fns and "bann_net_train" in fns and len(fns) >= 40


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "rs-bann_amd", "csrc"), "-j4"])
    return ctypes.CDLL(LIB)


def test_library_exports_every_header_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_nm_exports_are_plain_c(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for f in header_functions():
        assert f in exported, f"{f} not exported with C linkage"


def test_python_binding_covers_header():
    import bann._lib as L
    assert set(L.SIGNATURES) == set(header_functions())


def test_version_callable_without_device(lib):
    lib.bann_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.bann_version()


def test_ctx_create_fails_cleanly_without_gpu(lib):
    """On a CPU-only box bann_ctx_create must return an error code, not crash."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    lib.bann_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    rc = lib.bann_ctx_create(0, ctypes.byref(h))
    assert rc < 0 and not h.value


def test_binding_raises_without_library(tmp_path):
    import bann._lib as L
    saved = L._lib
    L._lib = None
    try:
        with pytest.raises(L.BannLibraryError):
            L.load_library(str(tmp_path / "missing.so"))
    finally:
        L._lib = saved
