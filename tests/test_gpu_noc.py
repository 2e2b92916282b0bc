"""Parity of the HIP NoC models and the history-tree queue model with the
reference KAT / fixtures and the CPU oracle.  Bit-exact."""
import numpy as np
import pytest

from graphite_amd import config as C
from graphite_amd import backend as B
from oracle import pyoracle as po
from golden_util import manifest, load
from gpu_util import torch_dev, to_dev, to_np
from test_oracle_golden import KAT

pytestmark = pytest.mark.gpu
M = manifest()


def test_history_tree_kat_on_gpu():
    torch_dev()
    be = B.Backend(C.default_config(4))
    d = be.queue_delay_batch([t for t, _, _ in KAT], [p for _, p, _ in KAT])
    assert d.tolist() == [x for _, _, x in KAT]


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] == "htree"])
def test_history_tree_fixtures_on_gpu(name):
    torch_dev()
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 3)
    be = B.Backend(C.default_config(4, max_list_size=e["max_list_size"], analytical_enabled=int(e["analytical"])))
    np.testing.assert_array_equal(be.queue_delay_batch(rows[:, 0], rows[:, 1]), rows[:, 2])


@pytest.mark.parametrize("max_size", [2, 7, 64, 65, 100, 128, 129])
@pytest.mark.parametrize("analytical", [0, 1])
def test_history_tree_wave_op_matches_avl_on_random_streams(max_size, analytical):
    """gg_queue_delay_batch runs every request on a whole wave over an LDS image
    (HTree::delay_w, the coherent walkers' path; the one-lane HBM path beyond
    128 slots): delays equal the oracle's AVL restatement on request streams
    with backward jumps (mid-list inserts / erases, prunes, the M/G/1 branch)."""
    import ctypes
    torch_dev()
    L = po.lib()
    L.oracle_htree_create.restype = ctypes.c_void_p
    L.oracle_htree_create.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    L.oracle_htree_delay.restype = ctypes.c_uint64
    L.oracle_htree_delay.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
    L.oracle_htree_destroy.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(max_size * 2 + analytical)
    for min_proc in (1, 3, 13):
        n = 3000
        base, span, maxp, jump = 0, int(rng.integers(50, 4000)), int(rng.integers(min_proc, 40)), int(rng.integers(1, 30))
        t = np.zeros(n, np.uint64)
        p = rng.integers(1, maxp + 1, n).astype(np.uint64)
        for i in range(n):
            base += int(rng.integers(0, jump))
            t[i] = base - int(rng.integers(0, span)) if (rng.random() < 0.3 and base > span) else base
        be = B.Backend(C.default_config(4, max_list_size=max_size, analytical_enabled=analytical))
        got = be.queue_delay_batch(t, p, min_processing_time=min_proc)
        h = L.oracle_htree_create(min_proc, max_size, analytical)
        ref = np.array([L.oracle_htree_delay(h, int(a), int(b)) for a, b in zip(t, p)], np.uint64)
        L.oracle_htree_destroy(h)
        np.testing.assert_array_equal(got, ref, err_msg="min_proc %d" % min_proc)
        be.close()


def packets(T, n, seed, span_ps, self_frac=0.05):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, T, n).astype(np.uint32)
    dst = rng.integers(0, T, n).astype(np.uint32)
    self_m = rng.random(n) < self_frac
    dst[self_m] = src[self_m]
    bits = np.where(rng.random(n) < 0.5, C.shmem_modeled_bits(T, False),
                    C.shmem_modeled_bits(T, True)).astype(np.uint32)
    t = np.sort(rng.integers(0, span_ps, n)).astype(np.uint64)
    t[rng.random(n) < 0.1] += np.uint64(7)                          # some out-of-order times
    return src, dst, bits, t


def run_noc(torch, cfg, src, dst, bits, t, batches=1):
    be = B.Backend(cfg)
    n = len(src)
    outs = [np.zeros(n, np.uint64) for _ in range(3)]
    cuts = [n * k // batches for k in range(batches + 1)]
    for k in range(batches):
        sl = slice(cuts[k], cuts[k + 1])
        m = cuts[k + 1] - cuts[k]
        dev = [to_dev(torch, src[sl], torch.int32), to_dev(torch, dst[sl], torch.int32),
               to_dev(torch, bits[sl], torch.int32), to_dev(torch, t[sl], torch.int64)]
        o = [torch.zeros(m, dtype=torch.int64, device="cuda") for _ in range(3)]
        be.noc_route_batch(*dev, *o)
        torch.cuda.synchronize()
        for i in range(3):
            outs[i][sl] = to_np(o[i], np.uint64)
    return be, outs


def oracle_noc(cfg, src, dst, bits, t, batches=1):
    on = po.OracleNoc(cfg)
    n = len(src)
    outs = [np.zeros(n, np.uint64) for _ in range(3)]
    cuts = [n * k // batches for k in range(batches + 1)]
    for k in range(batches):
        sl = slice(cuts[k], cuts[k + 1])
        r = on.route(src[sl], dst[sl], bits[sl], t[sl])
        for i in range(3):
            outs[i][sl] = r[i]
    return on, outs


@pytest.mark.parametrize("T", [16, 64, 1024])
def test_hop_counter_matches_oracle(T):
    torch = torch_dev()
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER)
    src, dst, bits, t = packets(T, 50000, T, 10 ** 9)
    be, got = run_noc(torch, cfg, src, dst, bits, t)
    on, ref = oracle_noc(cfg, src, dst, bits, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())


@pytest.mark.parametrize("T,n,span,batches", [(16, 4000, 200000, 1), (64, 20000, 2000000, 2),
                                              (256, 30000, 1000000, 1), (64, 30000, 100000, 3),
                                              (16, 80000, 4000000, 1),      # chains beyond the sweep's LDS: general walk
                                              (1024, 131072, 50 * 131072, 1)])   # the bench batch's shape
def test_hop_by_hop_matches_oracle(T, n, span, batches):
    """gg_noc_route_batch under emesh_hop_by_hop: X / Y chains as position
    sweeps (k_chain_sweep), or the general serial walk for chains beyond its
    limits, bit-exact vs the oracle's global event queue."""
    torch = torch_dev()
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_BY_HOP)
    src, dst, bits, t = packets(T, n, T + n, span)
    be, got = run_noc(torch, cfg, src, dst, bits, t, batches)
    on, ref = oracle_noc(cfg, src, dst, bits, t, batches)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())
    assert int(ref[2].sum()) > 0                                   # contention was exercised


@pytest.mark.parametrize("max_size", [3, 129])
def test_hop_by_hop_list_sizes_match_oracle(max_size):
    """max_list_size 3 (the prune on almost every request, the M/G/1 branch
    often) and 129 (beyond the register queue: the general walk).  At 2 the
    M/G/1 branch reaches delays of ~1e16 cycles whose picosecond value
    overflows UInt64 (Latency::toPicosec's double -> UInt64 cast,
    time_types.h:81-90, is undefined there): outside the domain."""
    torch = torch_dev()
    cfg = C.default_config(64, net_model=C.NET_EMESH_HOP_BY_HOP, max_list_size=max_size)
    src, dst, bits, t = packets(64, 20000, 5 + max_size, 500000)
    be, got = run_noc(torch, cfg, src, dst, bits, t)
    on, ref = oracle_noc(cfg, src, dst, bits, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())


def test_hop_by_hop_without_queue_model():
    torch = torch_dev()
    cfg = C.default_config(64, net_model=C.NET_EMESH_HOP_BY_HOP, queue_model_enabled=0)
    src, dst, bits, t = packets(64, 5000, 3, 100000)
    be, got = run_noc(torch, cfg, src, dst, bits, t)
    on, ref = oracle_noc(cfg, src, dst, bits, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    assert int(ref[2].sum()) == 0


# ---- history_list / basic queue models (QueueModel::create, queue_model.cc:19-39) ----
def _qcfg(e, T=4):
    if e["kind"] == "qlist":
        return C.default_config(T, queue_model_type=C.QM_HISTORY_LIST, max_list_size=e["max_list_size"],
                                analytical_enabled=int(e["analytical"]), history_list_no_interleaving=e["aux"])
    return C.default_config(T, queue_model_type=C.QM_BASIC, basic_moving_avg=e["aux"])


@pytest.mark.parametrize("name", [k for k, v in M.items() if v["kind"] in ("qlist", "qbasic")])
def test_other_queue_model_fixtures_on_gpu(name):
    torch_dev()
    e = M[name]
    rows = load(e["file"], np.uint64).reshape(-1, 3)
    be = B.Backend(_qcfg(e))
    np.testing.assert_array_equal(be.queue_delay_batch(rows[:, 0], rows[:, 1]), rows[:, 2])


@pytest.mark.parametrize("qtype,aux,T,n,span", [
    (C.QM_HISTORY_LIST, 0, 16, 4000, 200000),
    (C.QM_HISTORY_LIST, 1, 64, 20000, 500000),             # interleaving disabled
    (C.QM_BASIC, 0, 64, 20000, 500000),                    # arithmetic mean over 64
    (C.QM_BASIC, C.MAVG_MEDIAN << 16 | 16, 16, 4000, 200000),
    (C.QM_BASIC, C.MAVG_NONE << 16, 256, 30000, 1000000),
])
def test_hop_by_hop_other_queue_models_match_oracle(qtype, aux, T, n, span):
    """Router output-port contention through network/emesh_hop_by_hop/queue_model/type
    = history_list / basic, bit-exact vs the oracle."""
    torch = torch_dev()
    kw = dict(basic_moving_avg=aux) if qtype == C.QM_BASIC else dict(history_list_no_interleaving=aux)
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_BY_HOP, queue_model_type=qtype, **kw)
    src, dst, bits, t = packets(T, n, T + n + qtype, span)
    be, got = run_noc(torch, cfg, src, dst, bits, t)
    on, ref = oracle_noc(cfg, src, dst, bits, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())
    assert int(ref[2].sum()) > 0


def test_unsupported_queue_model_is_rejected():
    torch_dev()
    with pytest.raises(Exception):
        B.Backend(C.default_config(16, net_model=C.NET_EMESH_HOP_BY_HOP, queue_model_type=C.QM_BASIC,
                                   basic_moving_avg=C.MAVG_GEOMETRIC_MEAN << 16))
