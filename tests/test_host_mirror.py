"""The C++ host mirror (graphite_amd/host/graphite_host.hpp): its sim.out-style
cache summary matches the reference's Cache::outputSummary text
(cache.cc:419-477), and its TraceReplayer drives the GPU backend to the
oracle's counters."""
import os
import subprocess

import numpy as np
import pytest

from graphite_amd import config as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPLAY = os.path.join(ROOT, "graphite_amd", "host", "gg_replay")


def reference_summary(name, c, write_back):
    """Cache::outputSummary (cache.cc:419-477), restated; float formatting is
    the default std::ostream one (6 significant digits, like %g)."""
    L = ["  Cache %s: " % name, "    Cache Accesses: %d" % c[0], "    Cache Misses: %d" % c[1]]
    L.append("    Miss Rate (%%): %s" % ("%g" % (100.0 * c[1] / c[0]) if c[0] else ""))
    L.append("      Read Accesses: %d" % c[2])
    L.append("      Read Misses: %d" % c[3])
    L.append("      Read Miss Rate (%%): %s" % ("%g" % (100.0 * c[3] / c[2]) if c[2] else ""))
    L.append("      Write Accesses: %d" % c[4])
    L.append("      Write Misses: %d" % c[5])
    if c[4]:
        L.append("      Write Miss Rate (%%): %g" % (100.0 * c[5] / c[4]))
    else:
        L.append("    Write Miss Rate (%): ")                 # the reference's 4-space quirk (cache.cc:445)
    L.append("    Evictions: %d" % c[6])
    if write_back:
        L.append("    Dirty Evictions: %d" % c[7])
    L += ["    Event Counters:", "      Tag Array Reads: %d" % c[8], "      Tag Array Writes: %d" % c[9],
          "      Data Array Reads: %d" % c[10], "      Data Array Writes: %d" % c[11]]
    return L


def test_summary_format_matches_reference():
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    out = subprocess.run([REPLAY, "--summary-selftest"], capture_output=True, text=True, check=True).stdout
    c1 = [1000, 250, 700, 150, 300, 100, 240, 0, 2600, 900, 760, 1250]
    c2 = [250, 180, 150, 110, 100, 70, 120, 45, 700, 600, 190, 480]
    exp = reference_summary("L1-D", c1, False) + reference_summary("L2", c2, True) + \
        reference_summary("L2", [0] * 12, True)
    assert out.splitlines() == exp


def parse_summaries(text):
    tiles = {}
    cur = None
    keys = {"Cache Accesses": 0, "Cache Misses": 1, "Read Accesses": 2, "Read Misses": 3, "Write Accesses": 4,
            "Write Misses": 5, "Evictions": 6, "Dirty Evictions": 7, "Tag Array Reads": 8,
            "Tag Array Writes": 9, "Data Array Reads": 10, "Data Array Writes": 11}
    for line in text.splitlines():
        s = line.strip()
        if s.startswith("Tile ") and s.endswith("Cache Summary:"):
            t = int(s.split()[1])
            tiles[t] = np.zeros((2, 12), np.uint64)
        elif s.startswith("Cache L1-D"):
            cur = 0
        elif s.startswith("Cache L2"):
            cur = 1
        elif ":" in s:
            k, v = s.split(":", 1)
            if k in keys and v.strip():
                tiles[t][cur, keys[k]] = int(v)
    return tiles


@pytest.mark.gpu
def test_trace_replayer_matches_oracle():
    from gpu_util import torch_dev
    torch_dev()
    from oracle import pyoracle as po
    T, N = 6, 30000
    out = subprocess.run([REPLAY, "--tiles", str(T), "--per-tile", str(N), "--lines-log2", "12", "--batches", "3"],
                         capture_output=True, text=True, check=True).stdout
    got = parse_summaries(out)
    a = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[0] for t in range(T)])
    m = np.concatenate([po.gen_uniform(t, 0, N, lines_log2=12)[1] for t in range(T)])
    oc = po.OracleCache(C.default_config(T))
    oc.run(a, m, np.arange(T + 1, dtype=np.uint64) * np.uint64(N))
    ref = oc.counters()
    for t in range(T):
        np.testing.assert_array_equal(got[t], ref[t])


def reference_net_summary(nc, f, hop_counter, hop_by_hop=False, contention=False):
    """NetworkModel::outputSummary (network_model.cc:274-316) + the hop counter's
    event counters (network_model_emesh_hop_counter.cc:226-236), restated;
    averages are float32 printed like %g."""
    import math
    f32 = lambda x: float(np.float32(x))
    L = ["    Total Packets Sent: %d" % nc["ps"], "    Total Flits Sent: %d" % nc["fs"],
         "    Total Bits Sent: %d" % nc["bs"], "    Total Packets Broadcasted: 0",
         "    Total Flits Broadcasted: 0", "    Total Bits Broadcasted: 0",
         "    Total Packets Received: %d" % nc["pr"], "    Total Flits Received: %d" % nc["fr"],
         "    Total Bits Received: %d" % nc["br"]]
    n = nc["pr"]
    if n:
        cyc = lambda ps: math.ceil(ps * f / 1.0e3)
        ns = lambda ps: math.ceil(ps / 1.0e3)
        avg = lambda v: "%g" % f32(f32(v) / np.float32(n))
        L += ["    Average Packet Latency (in clock cycles): " + avg(cyc(nc["lat"])),
              "    Average Packet Latency (in nanoseconds): " + avg(ns(nc["lat"])),
              "    Average Contention Delay (in clock cycles): " + avg(cyc(nc["con"])),
              "    Average Contention Delay (in nanoseconds): " + avg(ns(nc["con"]))]
    else:
        L += ["    Average Packet Latency (in clock cycles): 0", "    Average Packet Latency (in nanoseconds): 0",
              "    Average Contention Delay (in clock cycles): 0", "    Average Contention Delay (in nanoseconds): 0"]
    if hop_counter:
        L += ["    Event Counters:", "      Buffer Writes: %d" % nc["bw"], "      Buffer Reads: %d" % nc["brd"],
              "      Switch Allocator Traversals: %d" % nc["sa"], "      Crossbar Traversals: %d" % nc["xb"],
              "      Link Traversals: %d" % nc["lt"]]
    if hop_by_hop:   # outputEventCountSummary / outputContentionModelsSummary (hop_by_hop.cc:436-486)
        L += ["    Event Counters:", "      Buffer Writes: %d" % nc["bw"], "      Buffer Reads: %d" % nc["brd"],
              "      Switch Allocator Requests: %d" % nc["sa"]] + \
             ["      Crossbar[%d] Traversals: %d" % (i, nc["xb"] if i == 1 else 0) for i in range(1, 6)] + \
             ["      Link Traversals: %d" % nc["lt"]]
        if contention:   # RouterModel averages over ports 0..4 (router_model.cc:145-215), float
            f32 = np.float32
            pk = nc["rpk"]
            d = f32(f32(nc["rcc"]) / f32(pk)) if pk else f32(0)
            u = f32(0)
            for a, b in zip(nc["util"], nc["last"]):
                u = f32(u + (f32(f32(a) / f32(b)) if b else f32(0)))
            u = f32(u / f32(5))
            an = f32(f32(f32(nc["an"]) * f32(100)) / f32(pk)) if pk else f32(0)
            L += ["    Contention Counters:", "      Average EMesh Router Contention Delay: %g" % d,
                  "      Average EMesh Router Link Utilization: %g" % u, "      Analytical Models Used (%%): %g" % an]
    return L


def test_network_summary_format_matches_reference():
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    out = subprocess.run([REPLAY, "--net-summary-selftest"], capture_output=True, text=True, check=True).stdout
    nc = dict(ps=70, fs=430, bs=24530, pr=66, fr=400, br=23000, lat=1234567, con=45001,
              bw=1720, brd=1720, sa=280, xb=1720, lt=1720)
    z = {k: 0 for k in nc}
    nc2 = dict(nc, rcc=913, rpk=280, an=3, util=[120, 0, 450, 77, 1000], last=[9000, 0, 12345, 8000, 40001])
    exp = reference_net_summary(nc, 1.0, True) + reference_net_summary(nc, 2.5, False, hop_by_hop=True) + \
        reference_net_summary(nc2, 1.0, False, hop_by_hop=True, contention=True) + \
        reference_net_summary(z, 1.0, False)
    assert out.splitlines() == exp


def reference_dram_summary(st, queue_block):
    """DramPerfModel::outputSummary (dram_perf_model.cc:131-164), restated:
    double sums / count printed as float (0 accesses: x86 default NaN, "-nan");
    QueueModel::getQueueUtilization (queue_model.cc:57-62) and the analytical
    fraction in float."""
    f32 = np.float32
    g = lambda x: "-nan" if np.isnan(x) else "%g" % float(x)
    n = st["dram"]
    avg = lambda s: g(f32(s / n) if n else float("nan"))
    L = ["Dram Performance Model Summary: ", "    Total Dram Accesses: %d" % n,
         "    Average Dram Access Latency (in nanoseconds): " + avg(st["lat"]),
         "    Average Dram Contention Delay (in nanoseconds): " + avg(st["qd"])]
    if queue_block:
        util = f32(f32(st["util"]) / f32(st["last"])) if st["last"] else f32(0)
        frac = f32(f32(st["an"]) / f32(st["qreq"]))
        L += ["    Queue Model:", "      Queue Utilization(%%): %s" % g(f32(util * f32(100))),
              "      Analytical Model Used(%%): %s" % g(f32(frac * f32(100)))]
    return L


def reference_directory_summary(st, auto):
    """"Dram Directory Summary:" + DirectoryCache::outputSummary
    (memory_manager.cc:427-428, directory_cache.cc:350-369,385-398); auto =
    (entries, size KB, access cycles) when "auto", else None."""
    L = ["Dram Directory Summary:"]
    if auto:
        L += ["    Total Entries [auto-generated]: %d" % auto[0], "    Size (in KB) [auto-generated]: %d" % auto[1],
              "    Access Time (in clock cycles) [auto-generated]: %d" % auto[2]]
    return L + ["    Total Accesses: %d" % st["dacc"], "    Total Evictions: %d" % st["dev"],
                "    Total Back-Invalidations: %d" % st["dbi"]]


def test_memory_summary_format_matches_reference():
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    out = subprocess.run([REPLAY, "--mem-summary-selftest"], capture_output=True, text=True, check=True).stdout
    st = dict(dacc=5123, dev=17, dbi=9, dram=321, lat=40417, qd=1537, qreq=321, an=7, util=4173, last=90211)
    z = {k: 0 for k in st}
    c1 = [1000, 250, 700, 150, 300, 100, 240, 0, 2600, 900, 760, 1250]
    c2 = [250, 180, 150, 110, 100, 70, 120, 45, 700, 600, 190, 480]
    # SURVEY.md §8 derived constants: 64 tiles -> 1024x16 entries, 128 KB, 6 cycles;
    # 1024 tiles -> 2 MB, 16 cycles
    exp = ["Cache Summary:"] + reference_summary("L1-D", c1, False) + reference_summary("L2", c2, True) + \
        reference_dram_summary(st, True) + reference_directory_summary(st, (16384, 128, 6)) + \
        reference_dram_summary(st, True) + reference_directory_summary(z, (16384, 2048, 16)) + \
        reference_dram_summary(z, False) + reference_directory_summary(st, None) + \
        reference_dram_summary(st, False)
    assert out.splitlines() == exp


def reference_table(summaries):
    """TileManager::outputSummary's table (tile_manager_summary.cc:60-198),
    restated with std::string::find semantics (npos + 1 wraps to 0)."""
    def find(s, ch, pos):
        i = s.find(ch, pos) if pos <= len(s) else -1
        return i if i >= 0 else 2 ** 64 - 1

    def substr(s, pos, n):
        return s[pos:pos + n] if pos <= len(s) else None

    npos1 = lambda v: (v + 1) % 2 ** 64
    rows = summaries[0].count("\n") + 1
    cols = len(summaries) + 1
    cell = [[""] * cols for _ in range(rows)]
    s0, pos = summaries[0], 0
    for i in range(1, rows):                                  # addRowHeadings (:135-151)
        end = find(s0, ":", pos)
        cell[i][0] = substr(s0, pos, end - pos)
        pos = npos1(find(s0, "\n", pos))
    for i in range(cols - 1):                                 # addColHeadings (:153-161)
        cell[0][i + 1] = "Tile %d" % i
    for t, s in enumerate(summaries):                         # addTileSummary (:163-176)
        pos = npos1(find(s, ":", 0))
        for i in range(1, rows):
            end = find(s, "\n", pos)
            cell[i][t + 1] = substr(s, pos, end - pos)
            pos = npos1(find(s, ":", pos))
    w = [max(len(cell[r][c]) for r in range(rows)) for c in range(cols)]
    return "".join("".join(cell[r][c] + " " * (w[c] - len(cell[r][c])) + " | " for c in range(cols)) + "\n"
                   for r in range(rows))


def test_tile_summary_table_matches_reference(tmp_path):
    if not os.path.exists(REPLAY):
        pytest.skip("gg_replay not built")
    tiles = [
        "Cache Summary:\n  Cache L1-D: \n    Cache Accesses: 1000\n    Miss Rate (%): 25\nNetwork Summary: \n",
        "Cache Summary:\n  Cache L1-D: \n    Cache Accesses: 7\n    Miss Rate (%): 14.2857\nNetwork Summary: \n",
        "Cache Summary:\n  Cache L1-D: \n    Cache Accesses: 123456789\n    Miss Rate (%): \nNetwork Summary: \n",
        # not in "label: value" form: the reference's scanning drifts, and so must ours
        "no colon here\n  a: b: c\ntail: 1\n\nx: y\n",
    ]
    files = []
    for i, t in enumerate(tiles):
        f = tmp_path / ("t%d.txt" % i)
        f.write_text(t)
        files.append(str(f))
    for sel in (files[:3], files):
        out = subprocess.run([REPLAY, "--format-table"] + sel, capture_output=True, text=True, check=True).stdout
        assert out == reference_table([open(f).read() for f in sel])


@pytest.mark.parametrize("name", ["mosi_hot16", "mosi_hot16magic", "mosi_dir16", "mosi_fft10", "mosi_evict16", "mosi_evict16s4"])
def test_mosi_controller_summaries_match_reference(name):
    """The host mirror's MOSI blocks (writeMosiL2CntlrSummary /
    writeMosiDirectoryCntlrSummary) print the reference's own
    L2CacheCntlr::outputSummary + DramDirectoryCntlr::outputSummary text
    (…mosi/l2_cache_cntlr.cc:638-649, dram_directory_cntlr.cc:1041-1142, written
    by coh_harness_mosi) from the same event counters, byte for byte."""
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    out = subprocess.run([REPLAY, "--mosi-summary", os.path.join(g, "coh_%s_proto.u64" % name), "16"],
                         capture_output=True, text=True, check=True).stdout
    with open(os.path.join(g, "coh_%s_summary.txt" % name)) as f:
        assert out == f.read()
