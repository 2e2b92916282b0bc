"""emesh_hop_by_hop broadcast tree (network_model_emesh_hop_by_hop.cc:163-221):
the oracle restatement's properties on CPU, and gg_noc_route_tree (the HIP
global-order walk) bit-exact against it on the GPU.  The NoC oracle is
parity-unpinned (the router model cannot be compiled here); the
CPU tests pin the tree's zero-load shape from the reference's routing rules."""
import numpy as np
import pytest

from graphite_amd import config as C
from oracle import pyoracle as po

K = {n: i for i, n in enumerate(C.NET_COUNTERS)}


def _cfg(T, **kw):
    return C.default_config(T, net_model=C.NET_EMESH_HOP_BY_HOP, **kw)


def mixed_packets(T, n, seed, span_ps, bcast_frac=0.1):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, T, n).astype(np.uint32)
    dst = rng.integers(0, T, n).astype(np.uint32)
    self_m = rng.random(n) < 0.03
    dst[self_m] = src[self_m]
    dst[rng.random(n) < bcast_frac] = C.BROADCAST
    bits = np.where(rng.random(n) < 0.5, C.shmem_modeled_bits(T, False),
                    C.shmem_modeled_bits(T, True)).astype(np.uint32)
    t = np.sort(rng.integers(0, span_ps, n)).astype(np.uint64)
    t[rng.random(n) < 0.1] += np.uint64(7)
    return src, dst, bits, t


@pytest.mark.parametrize("T", [16, 64])
def test_lone_broadcast_zero_load_tree(T):
    """One broadcast on an idle mesh: every tile (the sender included) receives
    it after (XY distance + 1) router+link hops plus serialization; the
    router at c routes to 1 + its listed ports; counters add up."""
    cfg = _cfg(T)
    on = po.OracleNoc(cfg)
    w = int(np.floor(np.sqrt(T)))
    s = 2 * w + 1
    bits = 600
    (arr, zl, ct), (ba, bz, bc) = on.route_tree(np.array([s], np.uint32), np.array([C.BROADCAST], np.uint32),
                                                np.array([bits], np.uint32), np.array([1000], np.uint64))
    nf = -(-bits // cfg.flit_width)
    hop = (cfg.router_delay + cfg.link_delay) * 1000       # 1 GHz
    for c in range(T):
        d = abs(c % w - s % w) + abs(c // w - s // w)
        assert int(bz[0, c]) == (d + 1) * hop + nf * 1000
        assert int(bc[0, c]) == 0
        assert int(ba[0, c]) == 1000 + int(bz[0, c])
    nc = on.counters()
    assert nc[:, K["packets_received"]].tolist() == [1] * T
    assert int(nc[s, K["packets_broadcasted"]]) == 1 and int(nc[s, K["bits_broadcasted"]]) == bits
    assert int(nc[:, K["switch_alloc"]].sum()) == T                 # one router event per tile
    # tree edges + one SELF per tile: T - 1 links between routers + T ejections
    assert int(nc[:, K["link_traversals"]].sum()) == nf * (2 * T - 1)
    xb = [int(nc[:, K["crossbar"]].sum())] + [int(nc[:, K["crossbar%d" % m]].sum()) for m in range(2, 6)]
    assert sum(xb) == nf * T


def test_tree_walk_equals_unicast_walk_without_broadcasts():
    T = 64
    cfg = _cfg(T)
    src, dst, bits, t = mixed_packets(T, 6000, 5, 300000, bcast_frac=0.0)
    a = po.OracleNoc(cfg)
    ref = a.route(src, dst, bits, t)
    b = po.OracleNoc(cfg)
    got, _ = b.route_tree(src, dst, bits, t)
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(a.counters(), b.counters())
    assert int(ref[2].sum()) > 0


def test_broadcast_rejected_outside_hop_by_hop():
    on = po.OracleNoc(C.default_config(16, net_model=C.NET_EMESH_HOP_COUNTER))
    with pytest.raises(RuntimeError):
        on.route_tree(np.array([0], np.uint32), np.array([C.BROADCAST], np.uint32),
                      np.array([88], np.uint32), np.array([0], np.uint64))


# ---- GPU: gg_noc_route_tree vs the oracle ------------------------------------
def run_tree(torch, cfg, src, dst, bits, t, batches=1):
    from graphite_amd import backend as B
    from gpu_util import to_dev, to_np
    be = B.Backend(cfg)
    n, T = len(src), cfg.num_tiles
    outs = [np.zeros(n, np.uint64) for _ in range(3)]
    bouts = [[] for _ in range(3)]
    cuts = [n * k // batches for k in range(batches + 1)]
    for k in range(batches):
        sl = slice(cuts[k], cuts[k + 1])
        m = cuts[k + 1] - cuts[k]
        nb = int((dst[sl] == C.BROADCAST).sum())
        dev = [to_dev(torch, src[sl], torch.int32), to_dev(torch, dst[sl].view(np.int32), torch.int32),
               to_dev(torch, bits[sl], torch.int32), to_dev(torch, t[sl], torch.int64)]
        o = [torch.zeros(m, dtype=torch.int64, device="cuda") for _ in range(3)]
        bo = [torch.zeros(nb * T, dtype=torch.int64, device="cuda") for _ in range(3)]
        be.noc_route_tree(*dev, *o, *bo, nb)
        torch.cuda.synchronize()
        for i in range(3):
            outs[i][sl] = to_np(o[i], np.uint64)
            bouts[i].append(to_np(bo[i], np.uint64).reshape(nb, T))
    return be, outs, [np.concatenate(b) for b in bouts]


def oracle_tree(cfg, src, dst, bits, t, batches=1):
    on = po.OracleNoc(cfg)
    n = len(src)
    outs = [np.zeros(n, np.uint64) for _ in range(3)]
    bouts = [[] for _ in range(3)]
    cuts = [n * k // batches for k in range(batches + 1)]
    for k in range(batches):
        sl = slice(cuts[k], cuts[k + 1])
        o, b = on.route_tree(src[sl], dst[sl], bits[sl], t[sl])
        for i in range(3):
            outs[i][sl] = o[i]
            bouts[i].append(b[i])
    return on, outs, [np.concatenate(b) for b in bouts]


@pytest.mark.gpu
@pytest.mark.parametrize("T,n,span,batches,frac,qm", [(16, 3000, 200000, 1, 0.1, 1), (64, 4000, 400000, 2, 0.05, 1),
                                                      (64, 3000, 100000, 1, 0.02, 1), (16, 2000, 100000, 1, 0.2, 0),
                                                      (256, 2000, 400000, 1, 0.01, 1), (256, 3000, 600000, 1, 0.03, 1),
                                                      # the bench's mesh: 256 blocks x 4 routers
                                                      (1024, 3000, 400000, 1, 0.01, 1),
                                                      # more routers than the workgroup's threads
                                                      (2116, 1500, 400000, 1, 0.004, 1),
                                                      (4096, 1500, 400000, 1, 0.004, 1),
                                                      # beyond the windowed walk's LDS arrays: the serial walk
                                                      (4225, 600, 200000, 1, 0.01, 1)])
def test_broadcast_tree_matches_oracle_on_gpu(T, n, span, batches, frac, qm):
    from gpu_util import torch_dev
    torch = torch_dev()
    cfg = _cfg(T, queue_model_enabled=qm)
    src, dst, bits, t = mixed_packets(T, n, T + n + batches, span, bcast_frac=frac)
    be, got, bgot = run_tree(torch, cfg, src, dst, bits, t, batches)
    on, ref, bref = oracle_tree(cfg, src, dst, bits, t, batches)
    uni = dst != C.BROADCAST
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g[uni], r[uni])
    for g, r in zip(bgot, bref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())
    assert bref[0].shape[0] > 0
    if qm:
        assert int(bref[2].sum()) > 0                              # broadcast copies were contended


@pytest.mark.gpu
@pytest.mark.parametrize("T,n,qtype,max_list,analytical", [
    (64, 3000, C.QM_HISTORY_TREE, 3, 1),      # pruned every request, M/G/1 branch taken
    (64, 3000, C.QM_HISTORY_TREE, 8, 0),
    (256, 3000, C.QM_HISTORY_TREE, 100, 0),
    (64, 3000, C.QM_HISTORY_LIST, 16, 1),
    (64, 3000, C.QM_BASIC, 100, 1)])
def test_broadcast_tree_queue_models_on_gpu(T, n, qtype, max_list, analytical):
    """The windowed walk's port tasks (a history tree's in-order requests from
    registers, every other request on memory) under each queue model, short
    lists (every request prunes; out-of-order requests) and the M/G/1 branch."""
    from gpu_util import torch_dev
    torch = torch_dev()
    cfg = _cfg(T, queue_model_type=qtype, max_list_size=max_list, analytical_enabled=analytical)
    src, dst, bits, t = mixed_packets(T, n, 7 * T + max_list, 150000, bcast_frac=0.05)
    be, got, bgot = run_tree(torch, cfg, src, dst, bits, t)
    on, ref, bref = oracle_tree(cfg, src, dst, bits, t)
    uni = dst != C.BROADCAST
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g[uni], r[uni])
    for g, r in zip(bgot, bref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())
    assert int(bref[2].sum()) > 0


@pytest.mark.gpu
def test_tree_walk_equals_stage_pipeline_without_broadcasts():
    """A unicast-only batch through gg_noc_route_tree (global-order walk) equals
    gg_noc_route_batch (independent X / Y chain stages) bit for bit."""
    from gpu_util import torch_dev
    from test_gpu_noc import run_noc
    torch = torch_dev()
    cfg = _cfg(64)
    src, dst, bits, t = mixed_packets(64, 5000, 11, 300000, bcast_frac=0.0)
    be1, got1, _ = run_tree(torch, cfg, src, dst, bits, t)
    be2, got2 = run_noc(torch, cfg, src, dst, bits, t)
    for a, b in zip(got1, got2):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(be1.noc_counters(), be2.noc_counters())


@pytest.mark.gpu
@pytest.mark.parametrize("T,n,frac", [(16, 2000, 0.1), (256, 3000, 0.03)])
def test_serial_tree_walk_matches_oracle_on_gpu(T, n, frac, monkeypatch):
    """The one-lane form (heap in LDS at 16 tiles, in HBM at 256), used where
    the windowed form has no lookahead (router + link delay 0)."""
    from gpu_util import torch_dev
    torch = torch_dev()
    monkeypatch.setenv("GG_NOC_TREE_SERIAL", "1")
    cfg = _cfg(T)
    src, dst, bits, t = mixed_packets(T, n, 3 * T + n, 300000, bcast_frac=frac)
    be, got, bgot = run_tree(torch, cfg, src, dst, bits, t)
    on, ref, bref = oracle_tree(cfg, src, dst, bits, t)
    uni = dst != C.BROADCAST
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g[uni], r[uni])
    for g, r in zip(bgot, bref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())


@pytest.mark.gpu
def test_zero_delay_mesh_takes_serial_walk():
    from gpu_util import torch_dev
    torch = torch_dev()
    cfg = _cfg(16, router_delay=0, link_delay=0)
    src, dst, bits, t = mixed_packets(16, 1500, 77, 100000, bcast_frac=0.1)
    be, got, bgot = run_tree(torch, cfg, src, dst, bits, t)
    on, ref, bref = oracle_tree(cfg, src, dst, bits, t)
    for g, r in zip(bgot, bref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())


def _replay_route(tmp_path, T, net, src, dst, bits, t):
    import os
    import subprocess
    replay = os.path.join(os.path.dirname(__file__), "..", "graphite_amd", "host", "gg_replay")
    if not os.path.exists(replay):
        pytest.skip("gg_replay not built")
    rec = np.zeros((len(src), 6), np.uint32)
    rec[:, 0], rec[:, 1], rec[:, 2] = src, dst, bits
    rec[:, 4:6] = t.view(np.uint32).reshape(-1, 2)
    f = tmp_path / "pk.bin"
    rec.tofile(str(f))
    return subprocess.run([replay, "--tiles", str(T), "--net", net, "--route", str(f)], capture_output=True,
                          text=True, check=True, timeout=120).stdout.splitlines()


@pytest.mark.gpu
def test_host_mirror_route_packet_broadcast(tmp_path):
    """graphite_amd::NetworkModel::routePackets (the C++ mirror, via gg_replay
    --route) under emesh_hop_by_hop: one RECEIVE_TILE hop per unicast packet;
    a broadcast takes the tree, one hop per application tile, then a
    zero-latency hop per system tile (processCornerCases,
    network_model.cc:451-458); equal to the oracle, and the summaries'
    broadcast lines count them."""
    T = 16
    cfg = _cfg(T)
    src, dst, bits, t = mixed_packets(T, 600, 123, 60000, bcast_frac=0.05)
    out = _replay_route(tmp_path, T, "hop_by_hop", src, dst, bits, t)
    on = po.OracleNoc(cfg)
    (ra, rz, rc), (ba, bz, bc) = on.route_tree(src, dst, bits, t)
    exp, b = [], 0
    for k in range(len(src)):
        if dst[k] != C.BROADCAST:
            exp.append("%d %d %d %d" % (dst[k], ra[k], rz[k], rc[k]))
        else:
            exp += ["%d %d %d %d" % (c, ba[b, c], bz[b, c], bc[b, c]) for c in range(T)]
            exp += ["%d %d 0 0" % (c, t[k]) for c in (T, T + 1)]
            b += 1
    assert out[:len(exp)] == exp
    nc = on.counters()
    got_b = [int(x.split(":")[1]) for x in out[len(exp):] if x.startswith("    Total Packets Broadcasted:")]
    assert got_b == nc[:, K["packets_broadcasted"]].tolist() and sum(got_b) == b
    x2 = [int(x.split(":")[1]) for x in out[len(exp):] if x.startswith("      Crossbar[2] Traversals:")]
    assert x2 == nc[:, K["crossbar2"]].tolist()


@pytest.mark.gpu
def test_host_mirror_unrolls_broadcast_without_tree(tmp_path):
    """emesh_hop_counter has no broadcast capability: Network::netSend sends one
    unicast per tile (network.cc:187-195, the sender's own copy a zero-latency
    self packet), the system tiles zero-latency hops."""
    T = 16
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_COUNTER)
    src, dst, bits, t = mixed_packets(T, 300, 321, 60000, bcast_frac=0.1)
    out = _replay_route(tmp_path, T, "hop_counter", src, dst, bits, t)
    es, ed, eb, et, sys_after = [], [], [], [], []
    for k in range(len(src)):
        rcv = range(T) if dst[k] == C.BROADCAST else [dst[k]]
        for c in rcv:
            es.append(src[k]); ed.append(c); eb.append(bits[k]); et.append(t[k])
        sys_after.append(dst[k] == C.BROADCAST)
    on = po.OracleNoc(cfg)
    ra, rz, rc = on.route(np.array(es, np.uint32), np.array(ed, np.uint32), np.array(eb, np.uint32),
                          np.array(et, np.uint64))
    exp, i = [], 0
    for k in range(len(src)):
        n = T if sys_after[k] else 1
        exp += ["%d %d %d %d" % (ed[i + j], ra[i + j], rz[i + j], rc[i + j]) for j in range(n)]
        i += n
        if sys_after[k]:
            exp += ["%d %d 0 0" % (c, t[k]) for c in (T, T + 1)]
    assert out[:len(exp)] == exp


@pytest.mark.gpu
@pytest.mark.parametrize("T,n,frac", [(64, 3000, 0.05), (256, 3000, 0.03), (1024, 4000, 0.01)])
def test_one_workgroup_window_loop_matches_oracle_on_gpu(T, n, frac, monkeypatch):
    """The one-workgroup windowed form (GG_NOC_TREE_POOL=1, k_tree_pool; the
    default where the grid form's LDS does not fit, e.g. 4096 tiles) against
    the oracle: the same deliveries and counters as the grid form."""
    from gpu_util import torch_dev
    torch = torch_dev()
    monkeypatch.setenv("GG_NOC_TREE_POOL", "1")
    cfg = _cfg(T)
    src, dst, bits, t = mixed_packets(T, n, 5 * T + n, 300000, bcast_frac=frac)
    be, got, bgot = run_tree(torch, cfg, src, dst, bits, t)
    on, ref, bref = oracle_tree(cfg, src, dst, bits, t)
    uni = dst != C.BROADCAST
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(g[uni], r[uni])
    for g, r in zip(bgot, bref):
        np.testing.assert_array_equal(g, r)
    np.testing.assert_array_equal(be.noc_counters(), on.counters())
