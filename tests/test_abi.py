"""The C-ABI boundary: the engine library loads and exports every entry point
include/jylis_gpu.h declares (no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "jylis_gpu.h")
LIB = os.path.join(ROOT, "jylis_amd", "libjylis_gpu.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(jy_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "jylis_amd")], check=True)
    return C.CDLL(LIB)


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("jy_engine_create", "jy_gcount_converge", "jy_pncount_converge_block", "jy_treg_converge",
              "jy_tlog_converge", "jy_ujson_converge", "jy_keys_intern", "jy_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"declared in include/jylis_gpu.h but not exported: {missing}"


def test_python_binding_covers_the_header():
    from jylis_amd import _lib
    assert set(declared_symbols()) == set(_lib.SIGNATURES)


def test_host_mirror_symbols(lib):
    """include/jylis_host.h (the C++ Database / RepoManagerCore mirror)"""
    from jylis_amd import _lib
    text = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "jylis_host.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(jyh_[a-z0-9_]+)\s*\(", text)))
    assert syms and set(syms) == set(_lib.HOST_SIGNATURES)
    assert all(hasattr(lib, s) for s in syms)


def test_no_gpu_fails_loudly():
    """Without a GPU the engine refuses to start: no silent CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from jylis_amd.engine import Engine, EngineError
    with pytest.raises(EngineError):
        Engine(device=0)


def test_key_owner_is_host_pure(lib):
    from jylis_amd.engine import key_owner
    owners = [key_owner(f"k{i}", 8) for i in range(4000)]
    assert set(owners) == set(range(8))
    counts = [owners.count(s) for s in range(8)]
    assert min(counts) > 400  # roughly uniform
    assert key_owner("k1", 8) == key_owner(b"k1", 8)
