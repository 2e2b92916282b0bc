"""configs[4] coherent stress workload: the
oracle's generator (oracle_gen_stress, the checker of gg_gen_stress_trace)
has the stated shape — WRITE 1/2, 30 % of accesses to a 4096-line shared
pool, each pool line shared by a hashed group of ~64 tiles — and a coherent
oracle run of it completes.  The device generator and the GPU runs are in
tests/test_gpu_coherent.py."""
import numpy as np

from graphite_amd import config as C
from oracle import pyoracle as po

POOL_BASE = 1 << 45


def test_stress_generator_shape():
    T, N = 4096, 512
    groups = T // 64
    a, m, o = po.gen_stress_trace(T, N)
    assert abs((m & 1).mean() - 0.5) < 0.01
    pool = a >= np.uint64(POOL_BASE)
    assert abs(pool.mean() - 77 / 256) < 0.01
    line = ((a[pool] - np.uint64(POOL_BASE)) // np.uint64(64)).astype(np.int64)
    assert line.max() < 4096
    tile = (np.nonzero(pool)[0] // N).astype(np.int64)
    # every pool access of a tile is to a line of its group; groups ~64 tiles
    grp_of_tile = np.full(T, -1)
    g = line % groups
    for t in np.unique(tile)[:512]:
        gs = np.unique(g[tile == t])
        assert len(gs) == 1
        grp_of_tile[t] = gs[0]
    # sharer degree: distinct tiles touching each pool line
    key = np.unique(line * T + tile)
    degree = np.bincount(key // T, minlength=4096)
    assert 48 <= degree.mean() <= 72, degree.mean()


def test_stress_private_lines_stay_private():
    a, m, o = po.gen_stress_trace(256, 200)
    priv = a < np.uint64(POOL_BASE)
    tile = np.repeat(np.arange(256, dtype=np.uint64), 200)
    assert np.array_equal(a[priv] >> np.uint64(26), tile[priv])


def test_stress_coherent_oracle_run():
    """256 tiles x 60 records, 16-way L2 (configs[4] geometry), shared pool
    with 64-tile sharer groups: the run finishes (no deadlock / assert) and
    writes to shared pool lines invalidate their sharers."""
    T, N = 256, 60
    a, m, o = po.gen_stress_trace(T, N)
    oc = po.OracleCoherent(C.default_config(T, l2_assoc=16))
    out = oc.run(a, m, o)
    st = oc.tile_stats()
    S = {n: i for i, n in enumerate(C.TILE_STATS)}
    assert st[:, S["accesses"]].sum() == T * N
    inv = st[:, S["sent_inv_req"]].sum()
    exreq = st[:, S["sent_ex_req"]].sum()
    assert inv > 0 and exreq > 0
    assert len(out) == T * N
