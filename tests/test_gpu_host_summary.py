"""GPU: the host mirror's sim.out writers on a real coherent run.  gg_replay
--coherent runs the MSI coherent mode through the C ABI (gg_coherent_run) and
prints every tile's memory block (MemoryManager::outputSummary,
msi/memory_manager.cc:415-430) and memory-network block (Network::outputSummary,
network.cc:79-89); the expected text is the reference's format restated in
tests/test_host_mirror.py, filled with the C oracle's statistics of the same
seeded trace."""
import os
import subprocess

import numpy as np
import pytest

from graphite_amd import config as C
from tests.test_host_mirror import (REPLAY, reference_summary, reference_dram_summary,
                                    reference_directory_summary, reference_net_summary)

pytestmark = pytest.mark.gpu


def _expected(T, N, net, hop_by_hop, shards=1):
    from oracle import pyoracle as po
    cfg = C.default_config(T, net_model=net, num_shards=shards)
    a, m, o = po.gen_trace(T, N, hot_lines=64)
    oc = po.OracleCoherent(cfg)
    oc.run(a, m, o)
    st, cc, nc = oc.tile_stats(), oc.cache_counters(), oc.net_counters()
    S = {n: i for i, n in enumerate(C.TILE_STATS)}
    K = {n: i for i, n in enumerate(C.NET_COUNTERS)}
    # DirectoryCache auto sizing (SURVEY.md §8 derived constants): 16 tiles -> 16384 entries, 32 KB, 2 cycles
    auto = {16: (16384, 32, 2), 64: (16384, 128, 6)}[T]
    L = []
    for t in range(T):
        s = st[t]
        d = dict(dacc=s[S["dir_accesses"]], dev=s[S["dir_evictions"]], dbi=s[S["dir_back_invalidations"]],
                 dram=s[S["dram_accesses"]], lat=s[S["dram_latency_ns"]], qd=s[S["dram_queue_delay_ns"]],
                 qreq=s[S["dram_queue_requests"]], an=s[S["dram_queue_analytical"]],
                 util=s[S["dram_queue_utilized_ns"]], last=s[S["dram_queue_last_ns"]])
        d = {k: int(v) for k, v in d.items()}
        n = nc[t]
        g = lambda k: int(n[K[k]])
        nd = dict(ps=g("packets_sent"), fs=g("flits_sent"), bs=g("bits_sent"), pr=g("packets_received"),
                  fr=g("flits_received"), br=g("bits_received"), lat=g("total_latency_ps"),
                  con=g("total_contention_ps"), bw=g("buffer_writes"), brd=g("buffer_reads"), sa=g("switch_alloc"),
                  xb=g("crossbar"), lt=g("link_traversals"), rcc=g("router_contention_cycles"),
                  rpk=g("router_packets"), an=g("analytical_requests"),
                  util=[g("port%d_utilized_cycles" % p) for p in range(5)],
                  last=[g("port%d_last_cycles" % p) for p in range(5)])
        L += ["Tile %d Summary:" % t, "Cache Summary:"]
        L += reference_summary("L1-D", [int(x) for x in cc[t, 0]], False)
        L += reference_summary("L2", [int(x) for x in cc[t, 1]], True)
        L += reference_dram_summary(d, True) + reference_directory_summary(d, auto)
        # Network::outputSummary prints the static networks below SYSTEM: User (no traffic), Memory
        z = dict(ps=0, fs=0, bs=0, pr=0, fr=0, br=0, lat=0, con=0, bw=0, brd=0, sa=0, xb=0, lt=0, rcc=0, rpk=0, an=0,
                 util=[0] * 5, last=[0] * 5)
        L += ["Network Summary: ", "  Network (User): "]
        L += reference_net_summary(z, cfg.frequency_ghz, True, hop_by_hop=False, contention=False)
        L += ["  Network (Memory): "]
        L += reference_net_summary(nd, cfg.frequency_ghz, net == C.NET_EMESH_HOP_COUNTER,
                                   hop_by_hop=hop_by_hop, contention=hop_by_hop and bool(cfg.queue_model_enabled))
    return L


@pytest.mark.parametrize("T,N,net", [(16, 400, "hop_by_hop"), (16, 600, "hop_counter"), (64, 150, "hop_by_hop")])
def test_coherent_sim_out_matches_oracle(T, N, net):
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    out = subprocess.run([REPLAY, "--coherent", "--tiles", str(T), "--per-tile", str(N), "--hot-lines", "64",
                          "--net", net], capture_output=True, text=True, check=True, timeout=120).stdout
    netid = C.NET_EMESH_HOP_BY_HOP if net == "hop_by_hop" else C.NET_EMESH_HOP_COUNTER
    exp = _expected(T, N, netid, net == "hop_by_hop")
    got = out.splitlines()
    assert len(got) == len(exp)
    for i, (x, y) in enumerate(zip(got, exp)):
        assert x == y, "line %d: %r != %r" % (i, x, y)


def test_coherent_sim_out_over_rccl_ranks(tmp_path):
    """gg_replay's rank mode: an RCCL communicator (here of one rank, the
    only one a one-GPU box can form), the run by gg_coherent_run_ranks with
    gg_round_exchange at every quantum boundary: the sim.out of the 4-shard
    canonical schedule."""
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    T, N = 16, 300
    out = subprocess.run([REPLAY, "--coherent", "--tiles", str(T), "--per-tile", str(N), "--hot-lines", "64",
                          "--net", "hop_by_hop", "--shards", "4", "--ranks", "1", "--rank", "0",
                          "--id-file", str(tmp_path / "rccl.id")],
                         capture_output=True, text=True, check=True, timeout=120).stdout
    exp = _expected(T, N, C.NET_EMESH_HOP_BY_HOP, True, shards=4)
    got = out.splitlines()
    got = got[got.index("Tile 0 Summary:"):]          # RCCL prints its version banner on stdout first
    assert len(got) == len(exp)
    for i, (x, y) in enumerate(zip(got, exp)):
        assert x == y, "line %d: %r != %r" % (i, x, y)


@pytest.mark.gpu
def test_coherent_summary_table_matches_reference_layout():
    """gg_replay --table on a real coherent run: TileManager::outputSummary's
    table (tile_manager_summary.cc:135-244) of exactly the per-tile blocks the
    same run prints one by one."""
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    from tests.test_host_mirror import reference_table
    args = [REPLAY, "--coherent", "--tiles", "16", "--per-tile", "200", "--hot-lines", "64", "--net", "hop_by_hop"]
    blocks_txt = subprocess.run(args, capture_output=True, text=True, check=True, timeout=120).stdout
    table = subprocess.run(args + ["--table"], capture_output=True, text=True, check=True, timeout=120).stdout
    blocks, cur = [], None
    for line in blocks_txt.splitlines(keepends=True):
        if line.startswith("Tile ") and line.rstrip().endswith(" Summary:"):
            cur = []
            blocks.append(cur)
        else:
            cur.append(line)
    assert len(blocks) == 16
    assert table == reference_table(["".join(b) for b in blocks])


@pytest.mark.parametrize("table", [False, True])
def test_dump_summary_through_the_abi(table):
    """gg_dump_summary (the sim.out text through the C ABI, for callers that
    are not C++): the same blocks / table as the host mirror prints, against
    the reference format filled with the oracle's statistics."""
    import torch
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T, N = 16, 400
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_BY_HOP)
    a, m, o = po.gen_trace(T, N, hot_lines=64)
    be = B.Backend(cfg)
    be.coherent_run(torch.from_numpy(a.view(np.int64)).cuda(), torch.from_numpy(m.view(np.int32)).cuda(), o)
    torch.cuda.synchronize()
    txt = be.dump_summary(table=table)
    exp = _expected(T, N, C.NET_EMESH_HOP_BY_HOP, True)
    if not table:
        assert txt.splitlines() == exp
    else:
        from tests.test_host_mirror import reference_table
        blocks, cur = [], None
        for line in exp:
            if line.startswith("Tile ") and line.endswith(" Summary:"):
                cur = []
                blocks.append(cur)
            else:
                cur.append(line + "\n")
        assert txt == reference_table(["".join(b) for b in blocks])
    be.close()
