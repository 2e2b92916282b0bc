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
    assert B.load().gg_abi_version() == 10


def test_config_default_matches_python_mirror():
    from graphite_amd.config import GGConfig, default_config
    c = GGConfig()
    B.load().gg_config_default(ctypes.byref(c), 64)
    d = default_config(64)
    for f, _ in GGConfig._fields_:
        assert getattr(c, f) == getattr(d, f), f


def test_shard_map_abi_matches_python_and_oracle():
    """gg_shard_map (the reference's emesh_hop_by_hop process blocks,
    network_model_emesh_hop_by_hop.cc:367-433) == the Python mirror == the
    oracle's restatement, for square meshes and for the contiguous fallback."""
    import numpy as np
    from graphite_amd import config as C
    from oracle import pyoracle as po
    for T in (16, 32, 64, 100, 256, 1024, 4096):
        for K in (1, 2, 3, 4, 5, 6, 7, 8, 16):
            a = B.shard_map(T, K)
            np.testing.assert_array_equal(a, C.shard_map(T, K))
            np.testing.assert_array_equal(a, po.shard_map(T, K))
    # 1024 tiles in 8 shards: a 2 x 4 grid of 16 x 8 blocks
    m = B.shard_map(1024, 8).reshape(32, 32)
    assert (m[:8, :16] == 0).all() and (m[:8, 16:] == 1).all() and (m[24:, 16:] == 7).all()
