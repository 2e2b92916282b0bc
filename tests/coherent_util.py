"""Test helpers for the coherent mode: the oracle as a `graphite_amd.coherent`
engine (CPU), and the invariants every coherent run must satisfy."""
import numpy as np

from graphite_amd import config as C


class OracleEngine:
    """oracle.pyoracle.OracleCoherent behind the engine surface of
    graphite_amd.coherent.run (CPU tensors, for the gloo tests)."""

    def __init__(self, cfg, addr, meta, offs):
        from oracle import pyoracle as po
        self.cfg = cfg
        self.o = po.OracleCoherent(cfg)
        self.out = self.o.begin(addr, meta, offs)

    def quantum(self, q):
        return self.o.quantum(q)

    def export(self):
        import torch
        msgs = self.o.export(1 << 20)
        K = self.cfg.num_shards
        at = np.where(msgs["hop"] == C.HOP_NONE, msgs["dst"], msgs["hop"])
        shard = C.shard_map(self.cfg.num_tiles, K)[at]
        counts = np.bincount(shard, minlength=K)
        return torch.from_numpy(msgs.view(np.uint8).copy()), counts

    def import_(self, buf):
        b = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf)
        self.o.import_(np.frombuffer(b.tobytes(), dtype=C.CMSG_DTYPE))


def check_invariants(stats, cache, out, offs, per_tile_expected=None):
    """Size-independent properties of a finished coherent run."""
    T = stats.shape[0]
    S = {n: stats[:, i] for i, n in enumerate(C.TILE_STATS)}
    n = np.diff(np.asarray(offs, np.int64))
    if per_tile_expected is not None:
        assert np.array_equal(S["accesses"].astype(np.int64), n)
    assert np.array_equal(S["l1_hits"] + S["l2_hits"] + S["l2_misses"], S["accesses"])
    lvl = (out & 3).astype(np.int64)
    lat = out >> 2
    for t in range(T):
        seg = slice(int(offs[t]), int(offs[t + 1]))
        assert int(lat[seg].sum()) == int(S["latency_ps"][t])
        assert int((lvl[seg] == 0).sum()) == int(S["l1_hits"][t])
        assert int((lvl[seg] == 2).sum()) == int(S["l2_misses"][t])
    # L1-D accesses = trace records; L2 accesses = L1-D misses; L2 misses = directory requests
    assert np.array_equal(cache[:, 0, C.CACHE_COUNTERS.index("accesses")], S["accesses"])
    assert np.array_equal(cache[:, 1, C.CACHE_COUNTERS.index("accesses")],
                          cache[:, 0, C.CACHE_COUNTERS.index("misses")])
    assert np.array_equal(cache[:, 1, C.CACHE_COUNTERS.index("misses")], S["l2_misses"])
    reqs = S["sent_ex_req"] + S["sent_sh_req"]
    assert np.array_equal(reqs, S["l2_misses"])
    # every request gets one reply (MOSI: an UPGRADE_REP for a lone sharer / owner)
    reps = S["sent_ex_rep"].sum() + S["sent_sh_rep"].sum() + S["sent_upgrade_rep"].sum()
    assert reps == reqs.sum()
    assert S["msgs_sent"].sum() == S["msgs_received"].sum()
