"""Loader for the fixtures in tests/golden/ (written by oracle/ref/make_golden.sh
from the reference's own CacheSet / replacement policies / line-info classes,
IntervalTree and QueueModelMG1, compiled from /root/reference)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load(name, dtype):
    return np.fromfile(os.path.join(GOLDEN, name), dtype=dtype)


POLICY = {"lru": 0, "round_robin": 1}
