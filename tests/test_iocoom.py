"""The iocoom core model (IOCOOMCoreModel,
common/tile/core/models/iocoom_core_model.cc, carbon_sim.cfg's default core
type): an in-order core with a register scoreboard, a load queue and a store
buffer, over an instruction stream whose memory operands take their
latencies from an access stream (gg_iocoom_run).

CPU tests pin the C oracle (oracle_iocoom) against a Python loop written from
the reference functions (handleInstruction :66-227, executeLoad/Store
:140-165, LoadQueue::execute :182-208, StoreQueue::execute :250-284,
isAddressAvailable :296-309) on every [core/iocoom] switch, and the stream
checks.  GPU tests compare gg_iocoom_run with the oracle bit for bit, also
after a coherent run whose accesses the instructions consume.  Parity of this
row is pinned by the restatement only: the reference's core model needs
Boost, McPAT and a Pin instruction stream to run."""
import math

import numpy as np
import pytest

from graphite_amd import config as C

BARRIER, WRITE = 0xFFFFFFFF, 1


def py_iocoom(lq_n, sq_n, spec, rfo, ins, ins_offs, addr, meta, lat, acc_offs, f=1.0):
    one = int(math.ceil(1000.0 / f)) if f != 1.0 else 1000
    T = len(ins_offs) - 1
    out = np.zeros((T, C.NUM_IOCOOM_STATS), np.uint64)
    S = {n: i for i, n in enumerate(C.IOCOOM_STATS)}
    for t in range(T):
        st = [0] * C.NUM_IOCOOM_STATS
        sb, dep = [0] * 512, [0] * 512                       # scoreboard, unit (0 invalid, 1 load, 3 execution)
        lsb, lidx = [0] * lq_n, 0
        ssb, saddr, sidx = [0] * sq_n, [(1 << 64) - 1] * sq_n, 0
        curr, k = 0, int(acc_offs[t])
        for i in range(int(ins_offs[t]), int(ins_offs[t + 1])):
            r = ins[i]
            st[S["instructions"]] += 1
            if int(r["regs"]) & C.INS_SYNC:                 # a SyncInstruction: dynamic, cost = its stall
                assert int(meta[k]) == BARRIER
                stall = int(lat[k]); k += 1
                if stall == 0:
                    st[S["instructions"]] -= 1
                else:
                    curr += stall
                    st[S["sync_instructions"]] += 1
                    st[S["sync_stall_ps"]] += stall
                continue
            cost = int(math.ceil(1000.0 * int(r["cost"]) / f)) if f != 1.0 else 1000 * int(r["cost"])
            ready = curr
            nr, nw = int(r["regs"]) & 7, (int(r["regs"]) >> 3) & 7
            rl = re = ready
            for j in range(nr):
                g = int(r["reg"][j])
                if dep[g] == 1:
                    rl = max(rl, sb[g])
                elif dep[g] == 3:
                    re = max(re, sb[g])
            rr = max(rl, re)
            lqr = rmr = rr
            for _ in range(int(r["ops"]) & 3):              # memory read operands: executeLoad
                assert int(meta[k]) != BARRIER and not (int(meta[k]) & WRITE)
                a, L = int(addr[k]), int(lat[k]) + one
                st[S["data_accesses"]] += 1; st[S["data_latency_ps"]] += int(lat[k]); k += 1
                if any(saddr[q] == a and ssb[q] >= rr for q in range(sq_n)):
                    alloc, comp = rr, rr + one              # store-buffer bypass
                else:
                    alloc = max(lsb[lidx], rr)
                    last = (lidx + lq_n - 1) % lq_n
                    if spec:
                        comp = alloc + L
                        dl = max(comp, lsb[last] + one)
                    else:
                        comp = max(lsb[last], rr) + L
                        dl = comp
                    lsb[lidx] = dl
                    lidx = (lidx + 1) % lq_n
                lqr = max(lqr, alloc)
                rmr = max(rmr, comp)
            wor = rmr + cost
            smov = bool(int(r["ops"]) & C.INS_SIMPLE_MOV_LOAD)
            for j in range(nw):
                g = int(r["reg"][nr + j])
                sb[g] = wor
                dep[g] = 1 if smov else 3
            sqr = wor
            nwm = (int(r["ops"]) >> 2) & 3
            for _ in range(nwm):                            # memory write operands: executeStore
                assert int(meta[k]) != BARRIER and (int(meta[k]) & WRITE)
                a, L = int(addr[k]), int(lat[k]) + one
                st[S["data_accesses"]] += 1; st[S["data_latency_ps"]] += int(lat[k]); k += 1
                lld = lsb[(lidx + lq_n - 1) % lq_n]
                alloc = max(ssb[sidx], wor)
                lsd = ssb[(sidx + sq_n - 1) % sq_n]
                if rfo:
                    dl = max(alloc + L, lsd + one, lld)
                else:
                    dl = max(wor, lsd, lld) + L
                ssb[sidx], saddr[sidx] = dl, a
                sidx = (sidx + 1) % sq_n
                sqr = max(sqr, alloc)
            mem = ex = 0
            ex += re - ready; st[S["inter_exec_stall_ps"]] += re - ready
            mem += rr - re; st[S["inter_l1d_stall_ps"]] += rr - re
            mem += lqr - rr; st[S["load_queue_stall_ps"]] += lqr - rr
            curr = lqr
            if not smov:
                mem += rmr - lqr; st[S["intra_l1d_stall_ps"]] += rmr - lqr
                curr = rmr
                if nwm:
                    ex += wor - rmr; st[S["intra_exec_stall_ps"]] += wor - rmr
                    mem += sqr - wor; st[S["store_queue_stall_ps"]] += sqr - wor
                    curr = sqr
            if int(r["ops"]) & C.INS_ATOMIC:
                st[S["implicit_mfences"]] += 1
            if int(r["ops"]) >> C.INS_FENCE_SHIFT:
                st[S["explicit_fences"]] += 1
            st[S["memory_stall_ps"]] += mem
            st[S["execution_stall_ps"]] += ex
        assert k == int(acc_offs[t + 1])
        st[S["time_ps"]] = curr
        out[t] = st
    return out


def gen_streams(*args, **kw):
    from graphite_amd.backend import gen_iocoom_streams
    return gen_iocoom_streams(*args, **kw)


PARAMS = [(8, 8, 1, 1), (8, 8, 0, 0), (1, 1, 1, 0), (2, 3, 0, 1), (64, 64, 1, 1), (5, 7, 1, 1)]


@pytest.mark.parametrize("lq,sq,spec,rfo", PARAMS)
def test_oracle_iocoom_matches_reference_loop(lq, sq, spec, rfo):
    from oracle import pyoracle as po
    ins, io, addr, meta, lat, ao = gen_streams(4, 600, 7 + lq + 3 * sq + spec)
    for f in (1.0, 2.5):
        got = po.iocoom(C.IocoomParams(lq, sq, spec, rfo), ins, io, addr, meta, lat, ao, f)
        np.testing.assert_array_equal(got, py_iocoom(lq, sq, spec, rfo, ins, io, addr, meta, lat, ao, f))


def test_oracle_iocoom_store_bypass_and_dependences():
    """Hand-built cases, times at 1 GHz (1 cycle = 1000 ps):
    a store then a load of the same address (bypass: 1 cycle), a simple-mov
    load (the core moves on at allocation; the consumer waits on the LOAD
    unit), an ALU chain (execution-unit stalls)."""
    from oracle import pyoracle as po
    ins = np.zeros(5, C.INS_DTYPE)
    # 0: store r1 -> [A] (cost 1)      1: load [A] -> r2 (simple mov, cost 1)
    # 2: r3 = r2 * r2 (cost 3)         3: r4 = r3 + 1 (cost 1)      4: load [B] -> r5 (cost 1)
    ins[0] = (1, 1 << 2, 1 | (0 << 3), [1, 0, 0, 0, 0, 0])
    ins[1] = (1, 1 | C.INS_SIMPLE_MOV_LOAD, 0 | (1 << 3), [2, 0, 0, 0, 0, 0])
    ins[2] = (3, 0, 2 | (1 << 3), [2, 2, 3, 0, 0, 0])
    ins[3] = (1, 0, 1 | (1 << 3), [3, 4, 0, 0, 0, 0])
    ins[4] = (1, 1, 0 | (1 << 3), [5, 0, 0, 0, 0, 0])
    addr = np.array([0x40, 0x40, 0x80], np.uint64)
    meta = np.array([WRITE, 0, 0], np.uint32)
    lat = np.array([50000, 50000, 20000], np.uint64)
    io, ao = np.array([0, 5], np.uint64), np.array([0, 3], np.uint64)
    st = po.iocoom(C.IocoomParams(), ins, io, addr, meta, lat, ao)[0]
    S = {n: int(st[i]) for i, n in enumerate(C.IOCOOM_STATS)}
    # 0: no reads, wor = 0 + 1000, store allocates at 1000, curr = store_queue_ready = 1000;
    #    its buffer entry deallocates at max(1000 + 51000, 0 + 1000, 0) = 52000
    # 1: bypass (52000 >= 1000): completion 2000; r2 ready at 3000 (LOAD unit); curr = 1000
    # 2: waits for r2 on the LOAD unit: 3000; r3 = 6000 (EXECUTION unit); curr = 3000
    # 3: waits for r3 on the EXECUTION unit: 6000; curr = 6000
    # 4: a load queue miss at 6000: completion 6000 + 21000 = 27000; curr = 27000
    assert S["time_ps"] == 27000
    assert S["inter_l1d_stall_ps"] == 2000 and S["inter_exec_stall_ps"] == 3000
    assert S["intra_l1d_stall_ps"] == 21000 and S["intra_exec_stall_ps"] == 1000
    assert S["instructions"] == 5 and S["data_accesses"] == 3 and S["data_latency_ps"] == 120000
    assert S["memory_stall_ps"] == 2000 + 21000 and S["execution_stall_ps"] == 3000 + 1000


def test_oracle_iocoom_stream_errors():
    from oracle import pyoracle as po
    ins, io, addr, meta, lat, ao = gen_streams(2, 200, 3)
    p = C.IocoomParams()
    po.iocoom(p, ins, io, addr, meta, lat, ao)
    bad = meta.copy()
    k = int(np.nonzero(bad != BARRIER)[0][0])
    bad[k] ^= WRITE                                          # a read operand meets a write access
    with pytest.raises(ValueError):
        po.iocoom(p, ins, io, addr, bad, lat, ao)
    with pytest.raises(ValueError):                          # accesses left over
        po.iocoom(p, ins, io, np.append(addr, 0), np.append(meta, 0), np.append(lat, 0), ao + np.array([0, 0, 1], np.uint64))
    r = ins.copy()
    i = int(np.nonzero(((r["regs"] & C.INS_SYNC) == 0) & ((r["ops"] & 0xF) == 0))[0][0])
    r["regs"][i] = 1                                         # one read register, out of range
    r["reg"][i, 0] = 512
    with pytest.raises(ValueError):
        po.iocoom(p, r, io, addr, meta, lat, ao)


def _gpu_iocoom(torch, B, cfg, p, ins, io, addr, meta, lat, ao):
    from tests.gpu_util import to_dev
    be = B.Backend(cfg)
    be.iocoom_run(p, torch.from_numpy(ins.view(np.uint8).copy()).cuda(), io, to_dev(torch, addr, torch.int64),
                  to_dev(torch, meta, torch.int32), to_dev(torch, lat, torch.int64), ao)
    st = be.iocoom_stats()
    return be, st


@pytest.mark.gpu
@pytest.mark.parametrize("lq,sq,spec,rfo", PARAMS)
@pytest.mark.parametrize("T,per_tile,regs", [(16, 3000, 24), (300, 500, 512), (1, 1, 4)])
def test_gpu_iocoom_matches_oracle(lq, sq, spec, rfo, T, per_tile, regs):
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev
    torch = torch_dev()
    ins, io, addr, meta, lat, ao = gen_streams(T, per_tile, 100 + T + lq, regs=regs)
    p = C.IocoomParams(lq, sq, spec, rfo)
    for f in (1.0, 2.0):
        be, st = _gpu_iocoom(torch, B, C.default_config(T, frequency_ghz=f), p, ins, io, addr, meta, lat, ao)
        np.testing.assert_array_equal(st, po.iocoom(p, ins, io, addr, meta, lat, ao, f))
        be.close()


@pytest.mark.gpu
def test_gpu_iocoom_long_streams():
    """1024 tiles x 20 000 instructions (the headline's tile count), empty
    tiles included, against the oracle."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev
    torch = torch_dev()
    T = 1024
    ins, io, addr, meta, lat, ao = gen_streams(T, 20000, 5, regs=64)
    io = io.copy(); io[5] = io[4]                            # tile 4 empty, tile 5 owns the old [4, 6)
    ao = ao.copy(); ao[5] = ao[4]
    p = C.IocoomParams()
    be, st = _gpu_iocoom(torch, B, C.default_config(T), p, ins, io, addr, meta, lat, ao)
    ref = po.iocoom(p, ins, io, addr, meta, lat, ao)
    np.testing.assert_array_equal(st, ref)
    assert st[4, 0] == 0
    be.close()


@pytest.mark.gpu
def test_gpu_iocoom_after_coherent_run():
    """End to end: a coherent run's access words give the latencies of the
    memory operands of an instruction stream built over its accesses (one
    load or store per access, ALU instructions and SyncInstructions between);
    the summary prints iocoom's detailed stall breakdown."""
    from graphite_amd import backend as B
    from oracle import pyoracle as po
    from tests.gpu_util import torch_dev, to_dev, to_np
    torch = torch_dev()
    T, N = 64, 300
    cfg = C.default_config(T, num_shards=8, net_model=C.NET_EMESH_HOP_COUNTER)
    a, m, o = po.gen_trace(T, N, hot_lines=32)
    be = B.Backend(cfg)
    addr, meta = to_dev(torch, a, torch.int64), to_dev(torch, m, torch.int32)
    out = torch.zeros(len(a), dtype=torch.int64, device="cuda")
    be.coherent_run(addr, meta, o, out)
    lat = to_np(out, np.uint64) >> np.uint64(2)
    rng = np.random.default_rng(3)
    ins_l, offs = [], [0]
    for t in range(T):
        for r in range(int(o[t]), int(o[t + 1])):
            for _ in range(int(rng.integers(0, 3))):             # ALU instructions
                x = np.zeros(1, C.INS_DTYPE)
                x["cost"], x["regs"] = 1, 2 | (1 << 3)
                x["reg"][0, :3] = rng.integers(0, 16, 3)
                ins_l.append(x)
            x = np.zeros(1, C.INS_DTYPE)
            if int(m[r]) == BARRIER:
                x["regs"] = C.INS_SYNC
            elif int(m[r]) & WRITE:
                x["cost"], x["ops"], x["regs"] = 1, 1 << 2, 1
                x["reg"][0, 0] = rng.integers(0, 16)
            else:
                x["cost"], x["ops"], x["regs"] = 1, 1 | C.INS_SIMPLE_MOV_LOAD, 1 << 3
                x["reg"][0, 0] = rng.integers(0, 16)
            ins_l.append(x)
        offs.append(len(ins_l))
    ins = np.concatenate(ins_l)
    io = np.array(offs, np.uint64)
    p = C.IocoomParams()
    be.iocoom_run(p, torch.from_numpy(ins.view(np.uint8).copy()).cuda(), io, addr, meta,
                  to_dev(torch, lat, torch.int64), o)
    st = be.iocoom_stats()
    np.testing.assert_array_equal(st, po.iocoom(p, ins, io, a, m, lat, o, cfg.frequency_ghz))
    S = C.IOCOOM_STATS
    assert (st[:, S.index("data_accesses")] == np.diff(o)).all()
    # overlapped loads: the core finishes no later than the simple model's serial clock
    assert (st[:, S.index("time_ps")] <= be.coherent_stats()[0][:, C.TILE_STATS.index("clock_ps")] +
            1000 * np.diff(io).astype(np.uint64)).all()
    text = be.dump_summary()
    assert text.count("Core Summary:") == T and "      Load Queue: " in text and "      Store Queue: " in text
    be.close()


@pytest.mark.gpu
def test_gpu_iocoom_errors():
    from graphite_amd import backend as B
    from tests.gpu_util import torch_dev, to_dev
    torch = torch_dev()
    ins, io, addr, meta, lat, ao = gen_streams(4, 300, 9)
    be = B.Backend(C.default_config(4))
    with pytest.raises(B.GGError):
        be.iocoom_stats()                                    # not run yet
    bad = meta.copy()
    k = int(np.nonzero(bad != BARRIER)[0][0])
    bad[k] ^= WRITE
    be.iocoom_run(C.IocoomParams(), torch.from_numpy(ins.view(np.uint8).copy()).cuda(), io,
                  to_dev(torch, addr, torch.int64), to_dev(torch, bad, torch.int32), to_dev(torch, lat, torch.int64), ao)
    with pytest.raises(B.GGError):
        be.iocoom_stats()                                    # the streams disagree

    def run(i_, lat_):
        be.iocoom_run(C.IocoomParams(), torch.from_numpy(i_.view(np.uint8).copy()).cuda(), io,
                      to_dev(torch, addr, torch.int64), to_dev(torch, meta, torch.int32),
                      to_dev(torch, lat_, torch.int64), ao)
        return be.iocoom_stats()
    run(ins, lat)                                            # clean
    r = ins.copy()
    i = int(np.nonzero(((r["regs"] & C.INS_SYNC) == 0) & ((r["ops"] & 0xF) == 0))[0][0])
    r["regs"][i] = 1                                         # one read register, out of range
    r["reg"][i, 0] = 512
    with pytest.raises(B.GGError):
        run(r, lat)
    # a register time of 2^62 ps or more does not fit the scoreboard entry
    # beside its unit (gg_core.hip, kTimeMask): flagged, not wrapped
    big = lat.copy()
    big[(meta != BARRIER) & ((meta & WRITE) == 0)] = np.uint64(1) << np.uint64(62)
    with pytest.raises(B.GGError):
        run(ins, big)
    run(ins, lat)                                            # the context recovers
    for d in (-1, 1):                                        # the last tile runs out of accesses / leaves one
        ao2 = ao.copy()
        ao2[-1] = ao2[-1] + np.uint64(d) if d > 0 else ao2[-1] - np.uint64(1)
        n2 = int(ao2[-1])
        a2, m2, l2 = (np.resize(x, n2) for x in (addr, meta, lat))
        if d > 0:
            m2[-1] = 0                                       # an extra read access
        be.iocoom_run(C.IocoomParams(), torch.from_numpy(ins.view(np.uint8).copy()).cuda(), io,
                      to_dev(torch, a2, torch.int64), to_dev(torch, m2, torch.int32), to_dev(torch, l2, torch.int64), ao2)
        with pytest.raises(B.GGError):
            be.iocoom_stats()
    run(ins, lat)
    with pytest.raises(B.GGError):
        be.iocoom_run(C.IocoomParams(65, 8), torch.from_numpy(ins.view(np.uint8).copy()).cuda(), io,
                      to_dev(torch, addr, torch.int64), to_dev(torch, meta, torch.int32),
                      to_dev(torch, lat, torch.int64), ao)
    be.close()
