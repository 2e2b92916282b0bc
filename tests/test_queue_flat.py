"""The GPU's history-tree queue keeps its free intervals as a flat sorted array
with a first-fit search (graphite_amd/csrc/gg_dev.h); the reference keeps them
in an AVL tree searched by IntervalTree::searchTree (interval_tree.cc:366-394,
queue_model_history_tree.cc:44-126).  The two agree because the free
intervals are disjoint, at least min_processing_time long and separated by
at least one busy cycle (every processing time >= 1).  This test restates the
flat model in Python and checks it against the oracle's AVL restatement on
random request streams, and against the reference's own history-tree fixtures
(tests/golden/htree_*, incl. the M/G/1 branch)."""
import ctypes
import math

import numpy as np
import pytest

MAX = (1 << 64) - 1


class FlatQueue:
    """QueueModelHistoryTree over a sorted interval list (gg_dev.h HTree::tree_delay)."""

    def __init__(self, min_proc, max_size, analytical):
        self.iv = [[0, MAX]]
        self.min_proc, self.max_size, self.analytical = min_proc, max_size, analytical
        self.sig_sq = self.sig = 0.0
        self.n = self.newest = self.analytical_requests = 0

    def _mg1(self):                                   # QueueModelMG1::computeQueueDelay
        if self.n == 0:
            return 0
        var = (self.sig_sq / self.n) - ((self.sig / self.n) * (self.sig / self.n))
        sr = 1.0 / (self.sig / self.n)
        ar = self.n / self.newest
        if ar >= sr:
            ar = 0.999 * sr
        return int(math.ceil(0.5 * sr * ar * ((1 / (sr * sr)) + var) / (sr - ar)))

    def delay(self, t, p):
        iv = self.iv
        if len(iv) >= self.max_size:
            iv.pop(0)                                 # prune the min node
        if self.analytical and iv[0][0] > t + p:
            self.analytical_requests += 1
            qd = self._mg1()
        else:
            i = next(i for i, (a, b) in enumerate(iv) if (a <= t and t + p <= b) or (a > t and b - a >= p))
            a, b = iv[i]
            if t >= a:
                qd = 0
                if t - a >= self.min_proc:
                    if b - (t + p) >= self.min_proc:
                        iv.insert(i + 1, [t + p, b])
                    iv[i][1] = t
                elif b - (t + p) >= self.min_proc:
                    iv[i][0] = t + p
                else:
                    iv.pop(i)
            else:
                qd = a - t
                if b - (a + p) >= self.min_proc:
                    iv[i][0] = a + p
                else:
                    iv.pop(i)
        self.sig_sq += float(p) * float(p)
        self.sig += float(p)
        self.n += 1
        self.newest = max(self.newest, t + qd + p)
        return qd


def _avl():
    from oracle import pyoracle as po
    L = po.lib()
    L.oracle_htree_create.restype = ctypes.c_void_p
    L.oracle_htree_create.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    L.oracle_htree_delay.restype = ctypes.c_uint64
    L.oracle_htree_delay.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    L.oracle_htree_analytical_requests.restype = ctypes.c_uint64
    L.oracle_htree_analytical_requests.argtypes = [ctypes.c_void_p]
    L.oracle_htree_destroy.argtypes = [ctypes.c_void_p]
    return L


@pytest.mark.parametrize("seed", range(6))
def test_flat_first_fit_equals_avl_search(seed):
    L = _avl()
    rng = np.random.default_rng(seed)
    for _ in range(12):
        min_proc = int(rng.integers(1, 15))
        max_size = int(rng.integers(2, 120))
        an = int(rng.integers(0, 2))
        h = L.oracle_htree_create(min_proc, max_size, an)
        f = FlatQueue(min_proc, max_size, an)
        base, span = 0, int(rng.integers(1, 5000))
        maxp, jump = int(rng.integers(1, 40)), int(rng.integers(1, 30))
        for _ in range(1500):
            base += int(rng.integers(0, jump))
            t = base - int(rng.integers(0, span)) if (rng.random() < 0.3 and base > span) else base
            p = int(rng.integers(1, maxp + 1))
            assert L.oracle_htree_delay(h, t, p) == f.delay(t, p)
        assert L.oracle_htree_analytical_requests(h) == f.analytical_requests
        L.oracle_htree_destroy(h)


def test_flat_matches_reference_history_tree_fixtures():
    import golden_util as G
    n_an = 0
    for name, e in G.manifest().items():
        if e["kind"] != "htree":
            continue
        rows = G.load(e["file"], np.uint64).reshape(-1, 3)
        f = FlatQueue(1, e["max_list_size"], e["analytical"])
        got = [f.delay(int(t), int(p)) for t, p in rows[:, :2]]
        np.testing.assert_array_equal(np.array(got, np.uint64), rows[:, 2], err_msg=name)
        assert f.analytical_requests == e["analytical_requests"], name
        n_an += f.analytical_requests
    assert n_an > 0, "no fixture reaches the M/G/1 branch"
