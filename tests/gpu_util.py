"""Helpers for the -m gpu tests (they call the HIP path through the C ABI)."""
import numpy as np
import pytest


def torch_dev():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def to_dev(torch, a, dtype):
    """numpy uint64/uint32 -> device int64/int32 with the same bits."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).to("cuda").to(dtype)


def to_np(t, dtype):
    return t.cpu().numpy().view(dtype)
