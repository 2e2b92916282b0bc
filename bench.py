#!/usr/bin/env python3
"""bench.py — simulated memory accesses per second of the MI355X backend.

Metric (BASELINE.json): "simulated mem accesses/sec (node) at 1024 tiles,
1/2/4/8 GPU; bit-exact stats".

Headline = the metric's configuration, BASELINE.json configs[3]: 1024 tiles
(32 x 32 mesh), the hotspot trace (80 % private lines, 20 % to 256 lines
shared by every tile, WRITE p = 1/3, ~2-cycle gaps), the full
pr_l1_pr_l2_dram_directory_msi protocol (L1-D / L2, full-map DRAM directory,
DRAM history-tree queue) on emesh_hop_by_hop with history-tree router
contention, lax-barrier quantum 1000 ns, 8 logical shards = the reference's
8-process 2-D blocks (network_model_emesh_hop_by_hop.cc:367-433).  The trace
is shortened to --per-tile accesses per tile (named in config.workload): the
configs[3] length (2^20) would take hours at this rate.  One step = one whole
coherent run of the workload from the reset state (every tile's trace to its
end), inputs resident in HBM.  With N GPUs each rank owns 8/N of the shards
and the held cross-shard records are exchanged at every quantum boundary;
the work is the same at every N ("strong" scaling) and the results are
bit-identical.

Reported with it: the roofline of the dominant kernel by device time
(k_c_walk: the X and Y walks are one kernel symbol) at SURVEY.md §8d's 16
algorithmic bytes per access (8 B address + 4 B meta in, 4 B result out),
accesses per launch from the run, the average launch duration measured live
in one extra untimed run: every launch stamps its first workgroup's start and
its last workgroup's end on the GPU's 100 MHz s_memrealtime clock (the span
rocprofv3's kernel trace reports; an event pair around a launch adds its
dispatch gap, ~7 %); the timed runs carry no instrumentation.  The C oracle on the
same workload as the CPU baseline, tile-parallel on the host's CPU share
(oracle_coh_set_threads) and on one thread; and a bit-exact check of every
output against the oracle in the same run.  Sections under their own keys:
the headline workload at 8x the trace length (coherent_long), the same
workload on emesh_hop_counter, configs[0] (captured FFT), the configs[1]
private-cache replay (round 1's headline), NoC batches and the configs[4]
stress geometry.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ALGO_BYTES_PER_ACCESS = 16     # Mode P: 8 B addr + 4 B meta in, 4 B result out
COH_BYTES_PER_ACCESS = 16      # Mode C: 8 B addr + 4 B meta in, 4 B result out
CORE_BYTES_PER_RECORD = 12     # core model: 4 B meta + 8 B access word in (per-tile sums out)
# Algorithmic bytes per access of each Mode P kernel
KERNEL_BYTES = {
    "cache_stream": 16,    # single pass (default): read addr (8) + meta (4), write result (4); state < 1%
    "cache_hist": 8,       # read addr (+ per-chunk set counts, scans: < 1%)
    "cache_scatter": 24,   # read addr + meta (12), write key (8) + record slot (4)
    "cache_replay": 12,    # read key (8), write result in slot order (4); state load/store < 1%
    "cache_unshard": 12,   # read slot (4) + result (4), write program-order result (4)
}
KERNEL_SYMBOL = {"cache_stream": "k_cache_stream", "cache_hist": "k_shard_hist", "cache_scatter": "k_shard_scatter",
                 "cache_replay": "k_cache_replay_lean", "cache_unshard": "k_unshard",
                 "coherent_step": "k_c_step", "coherent_walk": "k_c_walk", "coherent_persist": "k_c_persist"}
NET = {"hop_counter": 1, "hop_by_hop": 2, "magic": 0}


def pmc_traffic(kernel, key):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary
    (profiles/<round>/summary*.json, FETCH_SIZE / WRITE_SIZE in separate
    passes, calibrated per MI355X_MICROARCH.md; tools/pmc_summary.py) of the
    workload `key`, or None."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload_key") != key:
            continue
        ks = d.get("kernels", {})
        # the summary keys are rocprof's names (template arguments included)
        v = ks.get(kernel) or next((ks[k] for k in ks if k.split("<")[0].split("::")[-1] == kernel), None)
        if v and "hbm_bytes" in v:
            best = {"bytes": v["hbm_bytes"], "source": os.path.relpath(f, ROOT)}
            if "traffic_factors" in v:
                best["factors"] = v["traffic_factors"]
    return best


# LDS peak: 256 B/clk/CU for the 16-B-per-lane ds_read_b128 the kernel issues
# (MI355X_MICROARCH.md memory hierarchy: 64-256 B/clk by instruction) x 256 CUs
# x 2.4 GHz
LDS_PEAK_GBS = 256 * 256 * 2.4


def pmc_lds(kernel, key):
    """LDS bytes per launch of `kernel` (SQ_INSTS_LDS_{LOAD,STORE,ATOMIC}_BANDWIDTH,
    64-B units, one PMC pass) from a committed summary of workload `key`."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "summary*.json"))):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload_key") != key:
            continue
        v = d.get("kernels", {}).get(kernel)
        if v and "lds_bytes" in v:
            best = {"bytes": v["lds_bytes"], "source": os.path.relpath(f, ROOT)}
    return best


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--tiles", type=int, default=1024, help="headline tiles (configs[3]: 1024)")
    p.add_argument("--per-tile", type=int, default=256, help="headline accesses per tile")
    p.add_argument("--hot-lines", type=int, default=256, help="shared hot lines (configs[3]: 256)")
    p.add_argument("--shards", type=int, default=8, help="logical shards (the 8-process blocks)")
    p.add_argument("--net", default="hop_by_hop", choices=sorted(NET), help="headline memory network model")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="CPU-baseline oracle threads (0 = the host CPU share: OMP_NUM_THREADS, else the affinity set)")
    p.add_argument("--long-per-tile", type=int, default=2048, help="coherent_long section: accesses per tile")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--no-kernel-profile", action="store_true",
                   help="skip the extra instrumented run (for an external rocprofv3 trace of the timed runs alone)")
    p.add_argument("--sections",
                   default="coherent_long,exchange,hop_counter,hotspot256,stress,fft,private,private_16way,noc,"
                           "core_model,iocoom",
                   help="extra sections at N = 1 (comma list; '' = none)")
    p.add_argument("--hc-per-tile", type=int, default=1024, help="hop_counter section: accesses per tile")
    p.add_argument("--h256-per-tile", type=int, default=1024, help="hotspot256 section (configs[2]): accesses per tile")
    p.add_argument("--private-per-tile", type=int, default=1 << 20)
    p.add_argument("--cpu-sample-tiles", type=int, default=480, help="private section: tile replays of its CPU sample")
    p.add_argument("--replay-kernel", type=int, default=0)
    p.add_argument("--stress-tiles", type=int, default=4096)
    p.add_argument("--stress-per-tile", type=int, default=64, help="configs[4] coherent stress: records per tile")
    p.add_argument("--private16-per-tile", type=int, default=1 << 18)
    p.add_argument("--noc-packets", type=int, default=1 << 18)
    p.add_argument("--noc-tiles", type=int, default=1024)
    p.add_argument("--core-tiles", type=int, default=1024, help="core_model section: tiles of the synthetic trace")
    p.add_argument("--core-per-tile", type=int, default=1 << 18, help="core_model section: records per tile")
    p.add_argument("--iocoom-tiles", type=int, default=1024, help="iocoom section: tiles")
    p.add_argument("--iocoom-per-tile", type=int, default=16384, help="iocoom section: instructions per tile")
    p.add_argument("--fft-m", type=int, default=20,
                   help="configs[0] section: the reference's FFT -p16 -m<m> (configs[0]: m=20; the trace build() "
                        "captures; m=14 is committed)")
    return p.parse_args()


def maybe_spawn(args):
    """--gpus N without a torchrun environment: start N ranks (one process per
    GPU) through torch.distributed.run before anything touches the GPU, and
    exit with their status."""
    if args.gpus <= 1 or "RANK" in os.environ:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def coherent_workload(T, N, H, dev, workload="hotspot"):
    import torch
    from graphite_amd import backend as B
    addr = torch.empty(T * N, dtype=torch.int64, device=dev)
    meta = torch.empty(T * N, dtype=torch.int32, device=dev)
    if workload == "stress":
        B.gen_stress_trace(addr, meta, 0, T, N, T)
    else:
        B.gen_hotspot_trace(addr, meta, 0, T, N, hot_lines=H)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    return addr, meta, offs


def cpu_share():
    """Threads of the host's CPU share: OMP_NUM_THREADS when set (the GPU box
    sets it to the CPUs it allots one GPU), else the process affinity set."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(int(env), aff) if env and env.isdigit() else aff)


def coherent_run(args, T, N, H, K, net, world, rank, dev, steps, warmup, verify, cpu, workload="hotspot", l2_assoc=8,
                 kernel_profile=True):
    """One measurement of Mode C: `warmup` untimed + `steps` timed whole runs,
    barrier + synchronize around the timed region, max over ranks; then (if
    kernel_profile) one untimed run with HIP events around every launch for
    the per-kernel averages."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    from graphite_amd import dist as D
    k0, k1 = CO.shard_range(rank, world, K)
    cfg = C.default_config(T, num_shards=K, shard_begin=k0, shard_end=k1, net_model=net, l2_assoc=l2_assoc)
    be = B.Backend(cfg)
    addr, meta, offs = coherent_workload(T, N, H, dev, workload)
    out = torch.zeros(T * N, dtype=torch.int64, device=dev)

    def step():
        if world == 1:
            be.coherent_run(addr, meta, offs, out)
        else:
            CO.run_rccl(be, addr, meta, offs, out)     # gg_coherent_run_ranks: the exchange in the C ABI (RCCL)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = D.max_over_ranks(time.perf_counter() - t0)
    st, cc, ri = be.coherent_stats()
    nc = be.noc_counters()
    kern = {}
    if kernel_profile:
        # HIP event pairs on the launch stream around every 16th launch of each
        # kernel (the pair also holds the launch's dispatch; in-kernel spans,
        # every_launch=True, hold only its execution)
        be.set_timing(True)
        c0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        prof_s = time.perf_counter() - c0
        be.set_timing(False)
        for name in ("coherent_step", "coherent_walk_x", "coherent_walk_y", "coherent_persist"):
            try:
                ms, n = be.kernel_stats(name)
            except Exception:
                continue
            if n:
                kern[name] = {"total_ms": ms, "launches": n, "avg_us": 1e3 * ms / n}
        # the X and Y walks are one kernel symbol (k_c_walk<true>) in rocprof
        wx, wy = kern.pop("coherent_walk_x", None), kern.pop("coherent_walk_y", None)
        if wx or wy:
            ms = sum(w["total_ms"] for w in (wx, wy) if w)
            n = sum(w["launches"] for w in (wx, wy) if w)
            kern["coherent_walk"] = {"total_ms": ms, "launches": n, "avg_us": 1e3 * ms / n,
                                     "x": wx, "y": wy}
        kern["_profile_run_seconds"] = prof_s
    res = {"value": T * N * steps / elapsed, "seconds_per_run": elapsed / steps, "elapsed": elapsed,
           "quanta": int(ri[C.RUN_INFO.index("quanta")]), "steps": int(ri[C.RUN_INFO.index("steps")]),
           "messages": int(ri[C.RUN_INFO.index("net_msgs")] + ri[C.RUN_INFO.index("self_msgs")]),
           "boundary_records": int(ri[C.RUN_INFO.index("boundary_msgs")]),
           "simulated_ns": int(st[:, 0].max()) // 1000, "kernels": kern}
    if world > 1:
        # every rank holds its own tiles' outputs: the node's totals for the check
        import torch.distributed as dist
        tot = [torch.from_numpy(x.view(np.int64).copy()).to(dev) for x in (st, cc, nc)]
        for x in tot + [out]:
            dist.all_reduce(x)
        st, cc, nc = [x.cpu().numpy().view(np.uint64).reshape(y.shape) for x, y in zip(tot, (st, cc, nc))]
    if rank == 0 and verify:
        from oracle import pyoracle as po
        a = addr.cpu().numpy().view(np.uint64)
        m = meta.cpu().numpy().view(np.uint32)
        ocfg = C.default_config(T, num_shards=K, net_model=net, l2_assoc=l2_assoc)
        threads = args.cpu_threads or cpu_share()
        oc = po.OracleCoherent(ocfg, threads=threads)
        c0 = time.perf_counter()
        ref = oc.run(a, m, offs)
        pdt = time.perf_counter() - c0
        got = out.cpu().numpy().view(np.uint64)
        res["bit_exact_checked"] = bool(np.array_equal(got, ref) and np.array_equal(st, oc.tile_stats()) and
                                        np.array_equal(cc, oc.cache_counters()) and
                                        np.array_equal(nc, oc.net_counters()))
        if not res["bit_exact_checked"]:
            print("bench.py: COHERENT BIT-EXACT CHECK FAILED", file=sys.stderr)
        if cpu:
            o1 = po.OracleCoherent(ocfg)
            c0 = time.perf_counter()
            ref1 = o1.run(a, m, offs)
            sdt = time.perf_counter() - c0
            res["bit_exact_checked"] = res["bit_exact_checked"] and bool(np.array_equal(ref1, ref))
            res["cpu_baseline"] = {
                "value": T * N / pdt, "unit": "accesses/s", "cores": threads, "kind": "port",
                "sample": "the whole workload once (%d tiles x %d accesses): oracle/gg_coherent.inc -O3, tile-parallel "
                          "steps (each step's tiles, then the hop-by-hop routing stage by stage: injection per source, "
                          "X per row, Y per column, SELF per destination) on %d OpenMP threads = the host CPU share, "
                          "%.2f s" % (T, N, threads, pdt),
                "one_thread": {"value": T * N / sdt, "cores": 1, "seconds": sdt},
                "host": host_info()}
    be.close()
    return res


def host_info():
    info = {"nproc": os.cpu_count(), "cpu_share": cpu_share(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                info["model"] = line.split(":", 1)[1].strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def coherent_long_section(args, dev):
    """The headline workload at --long-per-tile accesses per tile (8x the
    headline's trace): one warm-up-free timed run, bit-exact against the
    tile-parallel oracle — the rate past the cold-start phase."""
    from graphite_amd import config as C
    T, N, H, K = args.tiles, args.long_per_tile, args.hot_lines, args.shards
    r = coherent_run(args, T, N, H, K, NET[args.net], 1, 0, dev, 1, 0, not args.no_verify, False,
                     kernel_profile=False)
    r["workload"] = ("%d tiles x %d hotspot accesses (%d hot lines), MSI + DRAM + %s, %d logical shards: the headline "
                     "at %dx its trace length" % (T, N, H, args.net, K, N // max(1, args.per_tile)))
    r["unit"] = "accesses/s"
    return r


def exchange_section(args, dev):
    """The per-quantum cost of the multi-rank exchange (gg_round_exchange:
    grouped per-peer slot send / receive + one status all-gather over RCCL, one
    host sync) measured on one GPU: the headline workload through
    gg_coherent_run_ranks over a one-rank RCCL communicator against the
    device-driven single-context loop (gg_coherent_run); same results bit for
    bit (checked)."""
    import socket
    import torch
    import torch.distributed as dist
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from graphite_amd import coherent as CO
    if dist.is_initialized():
        return {"skipped": "a process group already exists"}
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, world_size=1, rank=0)
    try:
        T, N, H, K = args.tiles, args.per_tile, args.hot_lines, args.shards
        cfg = C.default_config(T, num_shards=K, net_model=NET[args.net])
        addr, meta, offs = coherent_workload(T, N, H, dev)
        res, outs = {}, {}
        for mode in ("single", "rccl", "single", "rccl"):        # the second of each is timed
            be = B.Backend(cfg)
            out = torch.zeros(T * N, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "rccl":
                CO.run_rccl(be, addr, meta, offs, out)
            else:
                be.coherent_run(addr, meta, offs, out)
            torch.cuda.synchronize()
            res[mode] = time.perf_counter() - t0
            ri = be.coherent_stats()[2]
            outs[mode] = out.cpu().numpy()
            quanta = int(ri[C.RUN_INFO.index("quanta")])
            be.close()
        same = bool(np.array_equal(outs["single"], outs["rccl"]))
        return {"workload": "the headline workload (%d tiles x %d accesses, %s, %d shards) on one GPU" % (T, N, args.net, K),
                "quanta": quanta, "single_context_seconds": res["single"], "rccl_one_rank_seconds": res["rccl"],
                "exchange_us_per_quantum": 1e6 * (res["rccl"] - res["single"]) / max(1, quanta),
                "bit_identical": same,
                "note": "one host sync per quantum: the round enqueues the quantum's steps (a batch sized from "
                        "the quanta before), the tail kernel (status + export), RCCL (peer slots, one all-gather "
                        "of the status words), commit + import and the words' copy; the single context runs the "
                        "quantum loop on the device with no sync, so the difference per quantum bounds the "
                        "round's fixed cost"}
    finally:
        dist.destroy_process_group()


def hop_counter_section(args, dev):
    """The headline workload at --hc-per-tile accesses per tile on
    emesh_hop_counter (closed-form routes, no router contention)."""
    from graphite_amd import config as C
    T, N, H, K = args.tiles, args.hc_per_tile, args.hot_lines, args.shards
    r = coherent_run(args, T, N, H, K, C.NET_EMESH_HOP_COUNTER, 1, 0, dev, 1, 0, not args.no_verify,
                     not args.no_cpu_baseline, kernel_profile=False)
    r["workload"] = ("%d tiles x %d hotspot accesses (%d hot lines), MSI + DRAM + emesh_hop_counter, %d logical shards"
                     % (T, N, H, K))
    r["unit"] = "accesses/s"
    return r


def hotspot256_section(args, dev):
    """configs[2]: 256 tiles (16x16), the hotspot trace with 64 hot lines,
    MSI + full-map directory + DRAM + emesh_hop_by_hop, one process (one
    logical shard), --h256-per-tile accesses per tile; bit-exact against the
    tile-parallel oracle, which is its CPU baseline."""
    from graphite_amd import config as C
    T, N = 256, args.h256_per_tile
    r = coherent_run(args, T, N, 64, 1, C.NET_EMESH_HOP_BY_HOP, 1, 0, dev, 1, 0, not args.no_verify,
                     not args.no_cpu_baseline, kernel_profile=False)
    r["workload"] = ("configs[2]: %d tiles (16x16) x %d hotspot accesses (64 hot lines), MSI + DRAM + "
                     "emesh_hop_by_hop, one process" % (T, N))
    r["unit"] = "accesses/s"
    return r


def fft_section(args, dev):
    """configs[0]: SPLASH-2 FFT on 16 tiles, simulated in Mode C (MSI directory
    + emesh_hop_counter) on the GPU; bit-exact against the C oracle, whose run
    is the CPU baseline.  The trace is the reference's own fft.C (-p16
    -m<fft_m>) captured by tools/fft_trace when that capture exists
    (graphite_amd.capture.REAL_FFT_TRACES: -m20 written by build(), else the
    committed -m14)."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from graphite_amd import capture as cp
    m, p = args.fft_m, 16
    path = cp.REAL_FFT_TRACES.get(m)
    if not (path and os.path.exists(path)):
        m, path = 14, cp.REAL_FFT_TRACES[14]          # the -m20 capture is written by build() only
    a, meta, offs, bars = cp.load_fft_trace(path)
    src = ("the reference's tests/benchmarks/fft/fft.C -p%d -m%d captured by tools/fft_trace "
           "(heap accesses, 1 cycle per access, %d BARRIER calls per thread as barrier records)" % (p, m, len(bars[0])))
    cfg = C.default_config(p, net_model=C.NET_EMESH_HOP_COUNTER)
    be = B.Backend(cfg)
    addr = torch.from_numpy(a.view(np.int64)).to(dev)
    mt = torch.from_numpy(meta.view(np.int32)).to(dev)
    out = torch.zeros(len(a), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    be.coherent_run(addr, mt, offs, out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st, cc, ri = be.coherent_stats()
    res = {"workload": "configs[0]: %s, %d threads = %d tiles, %d accesses, pr_l1_pr_l2_dram_directory_msi + "
                       "emesh_hop_counter" % (src, p, p, len(a)),
           "value": len(a) / dt, "unit": "accesses/s", "seconds": dt,
           "steps": int(ri[C.RUN_INFO.index("steps")]), "simulated_ns": int(st[:, 0].max()) // 1000}
    if not args.no_verify:
        from oracle import pyoracle as po
        oc = po.OracleCoherent(cfg)
        c0 = time.perf_counter()
        ref = oc.run(a, meta, offs)
        cdt = time.perf_counter() - c0
        res["bit_exact_checked"] = bool(np.array_equal(out.cpu().numpy().view(np.uint64), ref) and
                                        np.array_equal(st, oc.tile_stats()) and
                                        np.array_equal(cc, oc.cache_counters()))
        if not res["bit_exact_checked"]:
            print("bench.py: FFT BIT-EXACT CHECK FAILED", file=sys.stderr)
        res["cpu_baseline"] = {"value": len(a) / cdt, "unit": "accesses/s", "cores": 1, "kind": "port",
                               "sample": "the whole FFT trace, oracle/gg_coherent.inc -O3, 1 thread, %.2f s" % cdt}
    be.close()
    return res


def noc_section(args, dev):
    """NetworkModel::routePacket batches (gg_noc_route_batch): uniform-random
    (src, dst) packets at configs[3]'s 1024-tile mesh, data-length messages
    (shmem EX_REP, 584 bits), injection times sorted, under emesh_hop_counter
    and emesh_hop_by_hop with history-tree router contention.  One batch per
    model, routed from fresh router queues, HIP-event timed, bit-exact
    against the C oracle (arrival, zero-load, contention and the per-tile
    counters), whose 1-thread run is the CPU baseline."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T = args.noc_tiles
    d = lambda x: torch.from_numpy(x.view(np.int64 if x.dtype == np.uint64 else np.int32)).to(dev)
    res = {"workload": "uniform-random packets of %d bits on the %d-tile mesh (configs[3]), one batch per model, "
                       "injection times ~50 ps apart" % (C.shmem_modeled_bits(T, True), T),
           "bytes_per_packet": 44,
           "bytes_per_packet_note": "44 B = this ABI's I/O (src, dst, bits u32; time u64 in; arrival, zero-load, "
                                    "contention u64 out); SURVEY.md section 8d's packed format is 24 B (GB_s_24)"}
    # the closed-form model is one thread per packet: a large batch; the hop-by-hop walk is serial per chain
    for name, model, n in (("hop_counter", C.NET_EMESH_HOP_COUNTER, 64 * args.noc_packets),
                           ("hop_by_hop", C.NET_EMESH_HOP_BY_HOP, args.noc_packets)):
        rng = np.random.default_rng(7)
        src = rng.integers(0, T, n).astype(np.uint32)
        dst = rng.integers(0, T, n).astype(np.uint32)
        bits = np.full(n, C.shmem_modeled_bits(T, True), np.uint32)
        t = np.sort(rng.integers(0, 50 * n, n)).astype(np.uint64)
        be = B.Backend(C.default_config(T, net_model=model))
        ins = [d(src), d(dst), d(bits), d(t)]
        outs = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(3)]
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        be.noc_route_batch(*ins, *outs)
        e1.record()
        torch.cuda.synchronize()
        dt = e0.elapsed_time(e1) / 1e3
        r = {"packets": n, "value": n / dt, "unit": "packets/s", "seconds": dt, "GB_s": 44 * n / dt / 1e9,
             "GB_s_24": 24 * n / dt / 1e9}
        if not args.no_verify:
            on = po.OracleNoc(C.default_config(T, net_model=model))
            c0 = time.perf_counter()
            ref = on.route(src, dst, bits, t)
            cdt = time.perf_counter() - c0
            r["bit_exact_checked"] = bool(all(np.array_equal(o.cpu().numpy().view(np.uint64), x)
                                              for o, x in zip(outs, ref)) and
                                          np.array_equal(be.noc_counters(), on.counters()))
            if not r["bit_exact_checked"]:
                print("bench.py: NOC %s BIT-EXACT CHECK FAILED" % name, file=sys.stderr)
            r["cpu_baseline"] = {"value": n / cdt, "unit": "packets/s", "cores": 1, "kind": "port",
                                 "sample": "the whole batch, oracle/gg_oracle.c -O3, 1 thread, %.2f s" % cdt}
        res[name] = r
        be.close()
    res["broadcast_tree"] = noc_tree_bench(args, dev, T)
    return res


def noc_tree_bench(args, dev, T):
    """gg_noc_route_tree: the hop-by-hop broadcast tree (hop_by_hop.cc:163-221) on
    the same mesh, 2 % of the packets broadcast (each reaches all T tiles), one
    global-order device walk; deliveries counted per (packet, receiving tile)."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    n = max(64, args.noc_packets // 16)
    rng = np.random.default_rng(9)
    src = rng.integers(0, T, n).astype(np.uint32)
    dst = rng.integers(0, T, n).astype(np.uint32)
    dst[rng.random(n) < 0.02] = C.BROADCAST
    nb = int((dst == C.BROADCAST).sum())
    bits = np.full(n, C.shmem_modeled_bits(T, True), np.uint32)
    t = np.sort(rng.integers(0, 50 * n, n)).astype(np.uint64)
    cfg = C.default_config(T, net_model=C.NET_EMESH_HOP_BY_HOP)
    be = B.Backend(cfg)
    d = lambda x: torch.from_numpy(x.view(np.int64 if x.dtype == np.uint64 else np.int32)).to(dev)
    ins = [d(src), d(dst), d(bits), d(t)]
    outs = [torch.zeros(n, dtype=torch.int64, device=dev) for _ in range(3)]
    bouts = [torch.zeros(nb * T, dtype=torch.int64, device=dev) for _ in range(3)]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    be.noc_route_tree(*ins, *outs, *bouts, nb)
    e1.record()
    torch.cuda.synchronize()
    dt = e0.elapsed_time(e1) / 1e3
    deliveries = (n - nb) + nb * T
    r = {"packets": n, "broadcasts": nb, "deliveries": deliveries, "value": deliveries / dt,
         "unit": "deliveries/s", "seconds": dt,
         "note": "k_tree_grid: conservative time windows of one router + link delay (a broadcast's shared port "
                 "delay couples the X and Y chains, so the unicast stage pipeline does not apply), one block per CU "
                 "owning its routers' queues in LDS, one grid barrier per window (DESIGN.md section 4b)"}
    if not args.no_verify:
        on = po.OracleNoc(cfg)
        c0 = time.perf_counter()
        (ra, rz, rc), (ba, bz, bc) = on.route_tree(src, dst, bits, t)
        cdt = time.perf_counter() - c0
        uni = dst != C.BROADCAST
        ok = all(np.array_equal(o.cpu().numpy().view(np.uint64)[uni], x[uni]) for o, x in zip(outs, (ra, rz, rc)))
        ok = ok and all(np.array_equal(o.cpu().numpy().view(np.uint64), x.reshape(-1)) for o, x in zip(bouts, (ba, bz, bc)))
        r["bit_exact_checked"] = bool(ok and np.array_equal(be.noc_counters(), on.counters()))
        if not r["bit_exact_checked"]:
            print("bench.py: NOC broadcast_tree BIT-EXACT CHECK FAILED", file=sys.stderr)
        r["cpu_baseline"] = {"value": deliveries / cdt, "unit": "deliveries/s", "cores": 1, "kind": "port",
                             "sample": "the whole batch, oracle/gg_oracle.c -O3, 1 thread, %.2f s" % cdt}
    be.close()
    return r


def stress_section(args, dev):
    """configs[4] coherent stress workload: 4096 tiles
    (64 x 64), 16-way L2 (512 sets), MSI + DRAM + emesh_hop_counter (the memory
    network of carbon_sim.cfg), 8 logical shards; the stress trace (WRITE p =
    1/2, 30 % of accesses to a 4096-line pool shared by ~64-tile groups) at
    --stress-per-tile records per tile.  One warm-up run, one timed; bit-exact
    against the all-core oracle, which is the CPU baseline with the 1-thread
    oracle beside it."""
    from graphite_amd import config as C
    T, N, K = args.stress_tiles, args.stress_per_tile, 8
    r = coherent_run(args, T, N, 0, K, C.NET_EMESH_HOP_COUNTER, 1, 0, dev, 1, 1, not args.no_verify,
                     not args.no_cpu_baseline, workload="stress", l2_assoc=16, kernel_profile=False)
    r["workload"] = ("configs[4]: %d tiles x %d stress accesses (WRITE p=1/2, 30%% to a 4096-line pool, ~64 sharers "
                     "per pool line), 16-way L2, MSI + DRAM + emesh_hop_counter, %d logical shards" % (T, N, K))
    r["unit"] = "accesses/s"
    return r


def private16_section(args, dev):
    """configs[4] cache geometry in Mode P (the private part): 4096 tiles,
    32KB/4w L1-D + 512KB/16w L2 (512 sets), 2^18 accesses per tile from the
    configs[1] uniform-random private generator (WRITE p = 1/3).  16-way L2
    sets do not fit the streaming kernel's LDS budget, so the batch runs the
    sharded path (shard scatter -> lean replay -> unshard).  HIP-event timed
    whole batch; one tile checked bit-exact against the oracle; the oracle on
    4 tiles, 1 thread, is the CPU baseline."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T, N = args.stress_tiles, args.private16_per_tile
    cfg = C.default_config(T, l2_assoc=16)
    be = B.Backend(cfg)
    be.set_timing(True)
    n = T * N
    addr = torch.empty(n, dtype=torch.int64, device=dev)
    meta = torch.empty(n, dtype=torch.int32, device=dev)
    result = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    B.gen_uniform_trace(addr, meta, 0, T, N, stream=stream)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    times = []
    for it in range(2):                       # first launch warms up
        be.reset()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        be.cache_access_batch(addr, meta, offs, result, None, stream)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / 1e3)
    dt = times[-1]
    kern = {k: be.kernel_time_ms(k) for k in KERNEL_BYTES}
    kern = {k: round(v, 4) for k, v in kern.items() if v >= 0}
    res = {"workload": "configs[4] private part: %d tiles x %d accesses, 32KB/4w L1-D + 512KB/16w L2, "
                       "configs[1] uniform-random private generator (WRITE p=1/3), Mode P" % (T, N),
           "value": n / dt, "unit": "accesses/s", "seconds": dt, "kernels_ms": kern,
           "path_GB_s": n * ALGO_BYTES_PER_ACCESS / dt / 1e9}
    if "cache_stream" in kern:                # the single-pass streaming replay (16-way form)
        gbs = n * ALGO_BYTES_PER_ACCESS / (kern["cache_stream"] / 1e3) / 1e9
        res["roofline"] = {"bound": "hbm", "kernel": "k_cache_stream", "achieved": gbs, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "bytes_per_access": ALGO_BYTES_PER_ACCESS,
                           "kernel_ms": kern["cache_stream"]}
    if not args.no_verify:
        t = T - 1
        a, m = po.gen_uniform(t, 0, N)
        oc = po.OracleCache(C.default_config(1, l2_assoc=16))
        ref = oc.run(a - np.uint64(t << 26), m, np.array([0, N], np.uint64))
        got = result[t * N:(t + 1) * N].cpu().numpy().view(np.uint32)
        res["bit_exact_checked"] = bool(np.array_equal(got, ref) and
                                        np.array_equal(be.cache_counters()[t], oc.counters()[0]))
        if not res["bit_exact_checked"]:
            print("bench.py: STRESS BIT-EXACT CHECK FAILED", file=sys.stderr)
        if not args.no_cpu_baseline:
            c0 = time.perf_counter()
            for k in range(4):
                a, m = po.gen_uniform(k, 0, N)
                po.OracleCache(C.default_config(1, l2_assoc=16)).run(a - np.uint64(k << 26), m,
                                                                       np.array([0, N], np.uint64))
            cdt = time.perf_counter() - c0
            res["cpu_baseline"] = {"value": 4 * N / cdt, "unit": "accesses/s", "cores": 1, "kind": "port",
                                   "sample": "4 tiles x %d accesses, oracle/gg_oracle.c -O3, 1 thread, %.2f s"
                                             % (N, cdt)}
    be.close()
    del addr, meta, result
    torch.cuda.empty_cache()
    return res


def core_model_section(args, dev):
    """§8f-4 core timing: gg_core_model_run (the simple core model over a
    coherent run's access words, a segmented reduction streamed from HBM at
    12 B per record: 4-B meta + 8-B access word).  (1) parity: a 64-tile
    hotspot coherent run, its core statistics bit-exact against the oracle and
    its completion times equal to the engine's clocks; (2) throughput: a
    synthetic trace of args.core_tiles x args.core_per_tile records (CONT runs
    included), HIP-event timed launch, 8 tiles checked against the oracle,
    which is the 1-thread CPU baseline on the same 8 tiles."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    res = {}
    cfg = C.default_config(64, num_shards=8, net_model=C.NET_EMESH_HOP_BY_HOP)
    a, m, o = po.gen_trace(64, 200, hot_lines=32)
    be = B.Backend(cfg)
    am = torch.from_numpy(m.view(np.int32)).to(dev)
    out = torch.zeros(len(a), dtype=torch.int64, device=dev)
    be.coherent_run(torch.from_numpy(a.view(np.int64)).to(dev), am, o, out)
    be.core_model_run(am, o, out)
    core = be.core_stats()
    clk = be.coherent_stats()[0][:, C.TILE_STATS.index("clock_ps")]
    parity = bool(np.array_equal(core, po.core_model(m, out.cpu().numpy().view(np.uint64), o, cfg.frequency_ghz)) and
                  np.array_equal(core[:, C.CORE_STATS.index("time_ps")], clk))
    be.close()
    T, N = args.core_tiles, args.core_per_tile
    n = T * N
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    gap = torch.randint(0, 64, (n,), device=dev, dtype=torch.int32, generator=g)
    wr = torch.randint(0, 2, (n,), device=dev, dtype=torch.int32, generator=g)
    cont = torch.rand(n, device=dev, generator=g) < 0.25
    cont.view(T, N)[:, 0] = False
    meta = torch.where(cont, torch.full_like(gap, -0x7FFFFFFF), (gap << 1) | wr)   # CONT | WRITE = 0x80000001
    acc = torch.randint(0, 1 << 40, (n,), device=dev, dtype=torch.int64, generator=g)
    del gap, wr, cont
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    be = B.Backend(C.default_config(T))
    be.set_timing(True)
    stream = torch.cuda.current_stream(dev)
    times = []
    for it in range(3):
        torch.cuda.synchronize()
        be.core_model_run(meta, offs, acc, stream)
        torch.cuda.synchronize()
        times.append(be.kernel_time_ms("core_model"))
    kms = min(times[1:])
    gbs = n * CORE_BYTES_PER_RECORD / (kms / 1e3) / 1e9
    core = be.core_stats()
    sample = list(range(0, T, max(1, T // 8)))[:8]
    ok, cdt = True, 0.0
    for t in sample:
        mm = meta[t * N:(t + 1) * N].cpu().numpy().view(np.uint32)
        aa = acc[t * N:(t + 1) * N].cpu().numpy().view(np.uint64)
        c0 = time.perf_counter()
        ref = po.core_model(mm, aa, np.array([0, N], np.uint64))
        cdt += time.perf_counter() - c0
        ok = ok and bool(np.array_equal(core[t], ref[0]))
    res = {"workload": "gg_core_model_run: synthetic %d tiles x %d records (25%% CONT line records), plus the "
                       "parity run (64-tile hotspot coherent run, hop-by-hop, 8 shards)" % (T, N),
           "value": n / (kms / 1e3), "unit": "records/s", "kernel_ms": kms,
           "roofline": {"bound": "hbm", "kernel": "k_core_model", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS, "bytes_per_record": CORE_BYTES_PER_RECORD},
           "bit_exact_checked": bool(ok and parity), "parity_run_exact": parity,
           "cpu_baseline": {"value": len(sample) * N / cdt, "unit": "records/s", "cores": 1, "kind": "port",
                            "sample": "%d tiles x %d records, oracle_core_model -O3, 1 thread, %.2f s"
                                      % (len(sample), N, cdt)}}
    if not res["bit_exact_checked"]:
        print("bench.py: CORE MODEL BIT-EXACT CHECK FAILED", file=sys.stderr)
    be.close()
    del meta, acc
    torch.cuda.empty_cache()
    return res


def iocoom_section(args, dev):
    """§8f-4 core timing, the iocoom model: gg_iocoom_run over synthetic
    instruction streams (random register operands from 64 registers, 0-2
    memory reads and 0-1 writes, simple-mov loads, SyncInstructions) of
    args.iocoom_tiles x args.iocoom_per_tile instructions at carbon_sim.cfg's
    [core/iocoom] defaults; HIP-event timed launch; every tile checked against
    the oracle, whose time on them is the 1-thread CPU baseline.  One wave
    per tile walks its instructions serially (register scoreboard, load
    queue, store buffer): the bound is that chain, not HBM (16 B per
    instruction + 20 B per access streamed)."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    T, N = args.iocoom_tiles, args.iocoom_per_tile
    ins, io, addr, meta, lat, ao = B.gen_iocoom_streams(T, N, 11, regs=64)
    p = C.IocoomParams()
    be = B.Backend(C.default_config(T))
    be.set_timing(True)
    d_ins = torch.from_numpy(ins.view(np.uint8)).to(dev)
    d_addr = torch.from_numpy(addr.view(np.int64)).to(dev)
    d_meta = torch.from_numpy(meta.view(np.int32)).to(dev)
    d_lat = torch.from_numpy(lat.view(np.int64)).to(dev)
    stream = torch.cuda.current_stream(dev)
    times = []
    for it in range(3):
        torch.cuda.synchronize()
        be.iocoom_run(p, d_ins, io, d_addr, d_meta, d_lat, ao, stream)
        torch.cuda.synchronize()
        times.append(be.kernel_time_ms("iocoom"))
    kms = min(times[1:])
    st = be.iocoom_stats()
    c0 = time.perf_counter()
    ref = po.iocoom(p, ins, io, addr, meta, lat, ao)
    cdt = time.perf_counter() - c0
    ok = bool(np.array_equal(st, ref))
    nbytes = 16 * len(ins) + 20 * len(addr)
    gbs = nbytes / (kms / 1e3) / 1e9
    res = {"workload": "gg_iocoom_run: synthetic %d tiles x %d instructions (%d accesses), [core/iocoom] defaults"
                       % (T, N, len(addr)),
           "value": len(ins) / (kms / 1e3), "unit": "instructions/s", "kernel_ms": kms,
           "roofline": {"bound": "latency", "kernel": "k_iocoom", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS,
                        "note": "bound by each tile's serial instruction chain (one wave per tile), not by HBM: "
                                "achieved / peak is the streamed bytes (16 per instruction + 20 per access) against "
                                "the HBM peak, reported for scale only"},
           "bit_exact_checked": ok,
           "cpu_baseline": {"value": len(ins) / cdt, "unit": "instructions/s", "cores": 1, "kind": "port",
                            "sample": "the same %d tiles x %d instructions, oracle_iocoom -O3, 1 thread, %.2f s"
                                      % (T, N, cdt)}}
    if not ok:
        print("bench.py: IOCOOM BIT-EXACT CHECK FAILED", file=sys.stderr)
    be.close()
    del d_ins, d_addr, d_meta, d_lat
    torch.cuda.empty_cache()
    return res


def cpu_baseline(tiles, per_tile, threads):
    """Oracle (oracle/gg_oracle.c, -O3) on a bounded sample: `tiles` tile
    replays (fresh cache state each) cycling over 16 pre-generated tiles of
    the same workload, one tile per thread at a time."""
    from graphite_amd import config as C
    from oracle import pyoracle as po
    traces = [po.gen_uniform(t, 0, per_tile) for t in range(min(16, tiles))]
    offs = np.array([0, per_tile], np.uint64)
    todo = list(range(tiles))
    lock = threading.Lock()

    def worker():
        while True:
            with lock:
                if not todo:
                    return
                t = todo.pop()
            oc = po.OracleCache(C.default_config(1))
            k = t % len(traces)
            a, m = traces[k]
            oc.run(a - np.uint64(k << 26), m, offs)   # tile k's private region, replayed as tile 0

    ths = [threading.Thread(target=worker) for _ in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    return tiles * per_tile / dt, dt


def private_section(args, dev, world=1, rank=0):
    """Mode P (round 1's headline): configs[1]'s uniform-random private trace at
    configs[3] scale (1024 tiles x --private-per-tile), single-pass streaming
    replay k_cache_stream; 3 timed replays; one tile bit-exact vs the oracle;
    the oracle on --cpu-sample-tiles tile replays as its CPU baseline.
    With N ranks (the path that shards with no data-path
    collective) rank r simulates global tiles [r*T, (r+1)*T) of the same
    generator (weak scaling, T = --tiles per GPU): each replay is bracketed by
    a barrier + synchronize, its time is the max over ranks, the per-tile
    counters are gathered and one tile of every rank is checked bit-exact."""
    import torch
    from graphite_amd import config as C
    from graphite_amd import backend as B
    from graphite_amd import dist as D
    T, N = args.tiles, args.private_per_tile
    t0g = rank * T                                    # this rank's first global tile
    cfg = C.default_config(T, replay_kernel=args.replay_kernel)
    be = B.Backend(cfg)
    be.set_timing(True)
    stream = torch.cuda.current_stream(dev)
    n = T * N
    addr = torch.empty(n, dtype=torch.int64, device=dev)
    meta = torch.empty(n, dtype=torch.int32, device=dev)
    result = torch.empty(n, dtype=torch.int32, device=dev)
    B.gen_uniform_trace(addr, meta, t0g, T, N, stream=stream)
    offs = np.arange(T + 1, dtype=np.uint64) * np.uint64(N)
    kms = {k: [] for k in KERNEL_BYTES}
    times = []
    for it in range(4):                               # the first replay warms up
        be.reset()
        torch.cuda.synchronize()
        D.barrier()
        t0 = time.perf_counter()
        be.cache_access_batch(addr, meta, offs, result, None, stream)
        torch.cuda.synchronize()
        dt = D.max_over_ranks(time.perf_counter() - t0)
        if it:
            times.append(dt)
            for k in KERNEL_BYTES:
                kms[k].append(be.kernel_time_ms(k))
    kern = {}
    for k, v in kms.items():
        v = [x for x in v if x >= 0]
        if v:
            ms = float(np.mean(v))
            kern[k] = {"ms": ms, "bytes_per_access": KERNEL_BYTES[k], "GB_s": n * KERNEL_BYTES[k] / (ms * 1e-3) / 1e9}
    dom = max(kern, key=lambda k: kern[k]["ms"])
    res = {"workload": "configs[1] uniform-random private generator at %d tiles x %d accesses%s, 32KB/4w L1-D + "
                       "512KB/8w L2, private-cache mode" % (T, N, " per GPU (global tiles [r*%d, (r+1)*%d) on rank r, "
                                                           "no data-path collective)" % (T, T) if world > 1 else ""),
           "value": world * n / float(np.mean(times)), "unit": "accesses/s", "n_gpus": world,
           "scaling": "weak", "seconds": float(np.mean(times)),
           "roofline": {"bound": "hbm", "kernel": KERNEL_SYMBOL[dom], "achieved": kern[dom]["GB_s"],
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": kern[dom]["GB_s"] / HBM_PEAK_GBS,
                        "kernel_ms": kern[dom]["ms"], "bytes_per_access": KERNEL_BYTES[dom], "kernels": kern}}
    prof = pmc_traffic(KERNEL_SYMBOL[dom], "private_%dx%d" % (T, N))
    res["roofline"]["traffic"] = prof["bytes"] if prof else None
    if prof:
        res["roofline"]["traffic_source"] = prof["source"]
    lds = pmc_lds(KERNEL_SYMBOL[dom], "private_%dx%d" % (T, N))
    if lds:
        # the kernel's LDS bytes per launch (PMC) over its live launch time
        gbs = lds["bytes"] / (kern[dom]["ms"] * 1e-3) / 1e9
        res["roofline"]["lds"] = {"achieved": gbs, "peak": LDS_PEAK_GBS, "unit": "GB/s", "frac": gbs / LDS_PEAK_GBS,
                                  "bytes_per_launch": lds["bytes"], "source": lds["source"]}
    if not args.no_verify:
        from oracle import pyoracle as po
        cnt = be.cache_counters()
        t = T - 1                                     # the rank's last tile, global id t0g + t
        a, m = po.gen_uniform(t0g + t, 0, N)
        oc = po.OracleCache(C.default_config(1))
        ref = oc.run(a - np.uint64((t0g + t) << 26), m, np.array([0, N], np.uint64))
        got = result[t * N:(t + 1) * N].cpu().numpy().view(np.uint32)
        ok = bool(np.array_equal(got, ref) and np.array_equal(cnt[t], oc.counters()[0]))
        full = D.gather_tile_counters(cnt, rank, world)           # [world * T, 2, 12], global tile order
        acc = full[:, 0, C.CACHE_COUNTERS.index("accesses")]
        ok = ok and bool(np.all(acc == np.uint64(N)))
        res["bit_exact_checked"] = D.max_over_ranks(0.0 if ok else 1.0) == 0.0
        res["counters_gathered"] = {"tiles": int(full.shape[0]), "l1d_accesses": int(acc.sum()),
                                    "l1d_misses": int(full[:, 0, C.CACHE_COUNTERS.index("misses")].sum())}
        if not res["bit_exact_checked"]:
            print("bench.py: PRIVATE BIT-EXACT CHECK FAILED", file=sys.stderr)
    if not args.no_cpu_baseline and world == 1:
        threads = args.cpu_threads or cpu_share()
        cps, cdt = cpu_baseline(args.cpu_sample_tiles, N, threads)
        res["cpu_baseline"] = {"value": cps, "unit": "accesses/s", "cores": threads, "kind": "port",
                               "sample": "%d tiles x %d accesses, oracle/gg_oracle.c -O3, one tile per thread, %.1f s"
                                         % (args.cpu_sample_tiles, N, cdt)}
    be.close()
    del addr, meta, result
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    maybe_spawn(args)
    # stdout carries the one JSON line only: libraries that print on stdout
    # (RCCL's version banner at communicator creation) go to stderr
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    from graphite_amd import config as C
    from graphite_amd import dist as D
    world, rank, local = D.env()
    if world != args.gpus and "RANK" in os.environ:
        args.gpus = world
    torch.cuda.set_device(local)
    D.init("nccl")
    dev = torch.device("cuda", local)
    net = NET[args.net]
    T, N, H, K = args.tiles, args.per_tile, args.hot_lines, args.shards
    if K % world:
        raise SystemExit("bench.py: %d logical shards do not split over %d ranks" % (K, world))
    head = coherent_run(args, T, N, H, K, net, world, rank, dev, args.steps, args.warmup,
                        not args.no_verify, world == 1 and not args.no_cpu_baseline,
                        kernel_profile=not args.no_kernel_profile)
    if rank == 0:
        kern = {k: v for k, v in head["kernels"].items() if not k.startswith("_")}
        dom = max(kern, key=lambda k: kern[k]["total_ms"]) if kern else None
        dk = kern.get(dom) if dom else None
        # accesses per launch of the dominant kernel x 16 B / its average launch time
        lacc = T * N / dk["launches"] if dk else None
        achieved = COH_BYTES_PER_ACCESS * lacc / (dk["avg_us"] * 1e-6) / 1e9 if dk else None
        wl = ("configs[3]: %d tiles (%dx%d mesh) x %d accesses per tile of the hotspot trace (20%% to %d lines "
              "shared by all tiles, WRITE p=1/3, ~2-cycle gaps), pr_l1_pr_l2_dram_directory_msi + full-map directory "
              "+ DRAM history-tree queue + %s (history-tree router contention), quantum 1000 ns, %d logical shards "
              "(2-D blocks) over %d GPU(s)" % (T, int(T ** 0.5), int(T ** 0.5), N, H,
                                              {1: "emesh_hop_counter", 2: "emesh_hop_by_hop", 0: "magic"}[net], K, world))
        out = {
            "metric": "simulated mem accesses/sec (node) at 1024 tiles, 1/2/4/8 GPU; bit-exact stats",
            "value": head["value"],
            "unit": "accesses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["seconds_per_run"] * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (configs[2..4] SplitMix64 hotspot trace, generated on device)",
            "config": {"workload": wl, "tiles": T, "accesses_per_tile": N, "hot_lines": H, "logical_shards": K,
                       "mode": "coherent", "network": args.net,
                       "parallelism": "%d logical shards over %d rank(s); held cross-shard records exchanged once "
                                      "per quantum%s" % (K, world, " (gg_coherent_run_ranks, RCCL)" if world > 1 else "")},
            "roofline": {"bound": "hbm", "kernel": KERNEL_SYMBOL.get(dom, dom), "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                         "traffic": None, "bytes_per_access": COH_BYTES_PER_ACCESS, "launch_accesses": lacc,
                         "kernel_avg_us": dk["avg_us"] if dk else None, "kernel_launches": dk["launches"] if dk else None,
                         "kernels": kern,
                         "timing": "HIP event pairs on the launch stream around every 16th launch of each "
                                   "kernel, one extra run; the timed runs carry no instrumentation",
                         "note": "Mode C is latency-bound: a step is a chain of dependent accesses per tile and each "
                                 "router port serves its packets one by one in the canonical order (DESIGN.md §4); "
                                 "the fraction measures how far that is from the HBM bound, not an HBM bottleneck"},
            "coherent": {k: head[k] for k in ("quanta", "steps", "messages", "boundary_records", "simulated_ns",
                                              "seconds_per_run")},
            "bit_exact_checked": head.get("bit_exact_checked"),
        }
        prof = pmc_traffic(KERNEL_SYMBOL.get(dom, dom), "coherent_%s_%dx%d_k%d" % (args.net, T, N, K))
        if prof:
            out["roofline"]["traffic"] = prof["bytes"]
            out["roofline"]["traffic_source"] = prof["source"]
            if "factors" in prof:
                out["roofline"]["traffic_factors"] = prof["factors"]
            out["roofline"]["traffic_note"] = ("HBM bytes per launch (FETCH_SIZE / WRITE_SIZE, calibrated at 8-B loads / "
                                               "scattered 4-B stores): router queue images and packet records read and "
                                               "written back per launch, the state SURVEY.md §8d excludes from the "
                                               "algorithmic bytes")
        if "cpu_baseline" in head:
            out["cpu_baseline"] = head["cpu_baseline"]
    # N > 1: the naturally sharding Mode P leg (private_section, weak scaling,
    # no data-path collective) beside the coherent headline
    secs = [x for x in args.sections.split(",") if x] if world == 1 else ["private"]
    t_sec = time.perf_counter()
    for name in secs:
        print("bench.py: section %s (%.0f s)" % (name, time.perf_counter() - t_sec), file=sys.stderr, flush=True)
        try:
            if name == "coherent_long" and args.long_per_tile:
                r = coherent_long_section(args, dev)
            elif name == "exchange":
                r = exchange_section(args, dev)
            elif name == "hop_counter":
                r = hop_counter_section(args, dev)
            elif name == "hotspot256" and args.h256_per_tile:
                r = hotspot256_section(args, dev)
            elif name == "fft" and args.fft_m:
                r = fft_section(args, dev)
            elif name == "private":
                r = private_section(args, dev, world, rank)
            elif name == "noc" and args.noc_packets:
                r = noc_section(args, dev)
            elif name == "stress" and args.stress_tiles:
                r = stress_section(args, dev)
            elif name == "private_16way" and args.stress_tiles:
                r = private16_section(args, dev)
            elif name == "core_model" and args.core_per_tile:
                r = core_model_section(args, dev)
            elif name == "iocoom" and args.iocoom_per_tile:
                r = iocoom_section(args, dev)
            else:
                continue
        except Exception as e:            # a section failing must not hide the headline
            r = {"error": repr(e)}
            print("bench.py: section %s failed: %r" % (name, e), file=sys.stderr)
        out[name] = r
    if rank == 0:
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if world > 1:
        D.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
