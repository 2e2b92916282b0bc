"""The C-ABI library loads and exports every symbol include/graphite_gpu.h
declares (no compute call: runs without a GPU)."""
import ctypes
import os
import re

from graphite_amd import backend as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "graphite_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)          # drop comments
    return sorted(set(re.findall(r"\b(gg_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(B.EXPORTS)


def test_library_exports_every_symbol():
    lib = ctypes.CDLL(B.LIB_PATH)
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert B.load().gg_abi_version() == 2


def test_config_default_matches_python_mirror():
    from graphite_amd.config import GGConfig, default_config
    c = GGConfig()
    B.load().gg_config_default(ctypes.byref(c), 64)
    d = default_config(64)
    for f, _ in GGConfig._fields_:
        assert getattr(c, f) == getattr(d, f), f


def test_capture_library_exports_every_symbol():
    from graphite_amd import capture as cp
    src = open(os.path.join(ROOT, "include", "graphite_capture.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    declared = sorted(set(re.findall(r"\b(gg_[a-z0-9_]+)\s*\(", src)))
    assert declared == sorted(cp.EXPORTS)
    lib = ctypes.CDLL(cp.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
