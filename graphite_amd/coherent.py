"""Coherent mode ("Mode C") across ranks: the lax-barrier quantum loop with the
per-quantum exchange of cross-shard ShmemMsgs.

The reference runs tiles in several processes that exchange every ShmemMsg
over its TCP transport in real time (common/transport/socktransport.cc) and
synchronise clocks at a lax barrier every quantum
(common/system/clock_skew_management_schemes/lax_barrier_sync_client.cc:31-69,
lax_barrier_sync_server.cc:57-160).  Here the tiles are split into logical
shards (the reference's 2-D process blocks of the mesh, config.shard_map, a
fixed part of the configuration); messages that stay inside a shard are
delivered step by step on the device, records that cross shards (messages, and
emesh_hop_by_hop packets at the edge of a shard's routers) are held until the
quantum boundary and exchanged there with one all-to-all (RCCL over xGMI on
GPUs, gloo on CPU).  The schedule — and so
every statistic — depends on the shard count, never on how many ranks hold the
shards.

`engine` is anything with the gg_coherent_* surface (graphite_amd.backend's
CoherentRun on a GPU; the oracle in the CPU tests):
  quantum(q) -> {"boundary_msgs", "min_next_ps", "active_tiles", "blocked_tiles", ...}
  export()   -> (uint8 tensor [n*64] on the engine's device, per-shard counts [num_shards])
  import_(uint8 tensor [m*64])
"""
import numpy as np

CMSG_BYTES = 64
NO_TIME = (1 << 64) - 1


def shard_range(rank, world, num_shards):
    """Logical shards owned by `rank`: [k0, k1).  num_shards must divide evenly."""
    if num_shards % world:
        raise ValueError("num_shards (%d) must be a multiple of the rank count (%d)" % (num_shards, world))
    per = num_shards // world
    return rank * per, (rank + 1) * per


def next_quantum(q, quantum_ps, msgs, active, blocked, min_next_ps):
    """Quantum to run after q, or None when the run is over (same rule as
    oracle_coh_run): with nothing in flight the empty quanta are skipped."""
    if active == 0 and msgs == 0:
        return None
    if msgs == 0 and blocked == 0:
        return max(q + 1, min_next_ps // quantum_ps)
    if msgs == 0 and blocked != 0:
        raise RuntimeError("coherent run deadlocked: tiles blocked with no message in flight")
    return q + 1


def run(engine, quantum_ps, num_shards, world=1, rank=0, backend=None, device="cpu"):
    """Run every quantum.  Returns the number of quanta executed."""
    import torch
    if world > 1:
        import torch.distributed as dist
    q, quanta = 0, 0
    per = num_shards // world
    while True:
        st = engine.quantum(q)
        quanta += 1
        buf, per_shard = engine.export()
        per_shard = np.asarray(per_shard, np.int64)
        if world == 1:
            if len(buf):
                engine.import_(buf)
            msgs, active, blocked, mn = (int(per_shard.sum()), st["active_tiles"], st["blocked_tiles"],
                                         st["min_next_ps"])
        else:
            send_counts = [int(per_shard[r * per:(r + 1) * per].sum()) for r in range(world)]
            cnt = torch.tensor(send_counts, dtype=torch.int64, device=device)
            rcv = torch.empty(world, dtype=torch.int64, device=device)
            dist.all_to_all_single(rcv, cnt)
            recv_counts = [int(x) for x in rcv.cpu().tolist()]
            home = buf.device
            send = buf if str(home) == str(torch.device(device)) else buf.to(device)   # gloo: stage through host
            out = torch.empty(sum(recv_counts) * CMSG_BYTES, dtype=torch.uint8, device=device)
            dist.all_to_all_single(out, send, [c * CMSG_BYTES for c in recv_counts],
                                   [c * CMSG_BYTES for c in send_counts])
            if len(out):
                engine.import_(out if out.device == home else out.to(home))
            tot = torch.tensor([int(per_shard.sum()), st["active_tiles"], st["blocked_tiles"]],
                               dtype=torch.int64, device=device)
            dist.all_reduce(tot)
            # min over ranks of an unsigned 64-bit time: shift into the signed range
            mnt = torch.tensor([st["min_next_ps"] - (1 << 63)], dtype=torch.int64, device=device)
            dist.all_reduce(mnt, op=dist.ReduceOp.MIN)
            msgs, active, blocked = [int(x) for x in tot.cpu().tolist()]
            mn = int(mnt.item()) + (1 << 63)
        nq = next_quantum(q, quantum_ps, msgs, active, blocked, mn)
        if nq is None:
            return quanta
        q = nq


def run_local(engines, quantum_ps, num_shards):
    """Several engines in one process (each owning an equal block of shards,
    in rank order), exchanging at the quantum boundary by direct copies —
    the same schedule as `run` over ranks.  Returns the number of quanta."""
    import torch
    world = len(engines)
    per = num_shards // world
    q, quanta = 0, 0
    while True:
        sts = [e.quantum(q) for e in engines]
        quanta += 1
        outs = [e.export() for e in engines]
        for r, e in enumerate(engines):
            parts = []
            for buf, counts in outs:
                counts = np.asarray(counts, np.int64)
                off = int(counts[:r * per].sum()) * CMSG_BYTES
                n = int(counts[r * per:(r + 1) * per].sum()) * CMSG_BYTES
                if n:
                    parts.append(buf[off:off + n].to(e.dev if hasattr(e, "dev") else "cpu"))
            if parts:
                e.import_(torch.cat(parts))
        msgs = sum(int(np.asarray(c, np.int64).sum()) for _, c in outs)
        active = sum(s["active_tiles"] for s in sts)
        blocked = sum(s["blocked_tiles"] for s in sts)
        mn = min(s["min_next_ps"] for s in sts)
        nq = next_quantum(q, quantum_ps, msgs, active, blocked, mn)
        if nq is None:
            return quanta
        q = nq


def rccl_comm_ptr(group=None):
    """The ncclComm_t (RCCL) of a torch.distributed "nccl" process group, as an
    int for the C ABI (created by a first collective if still lazy)."""
    import torch
    import torch.distributed as dist
    pg = group or dist.distributed_c10d._get_default_group()
    dev = torch.device("cuda", torch.cuda.current_device())
    t = torch.zeros(1, device=dev)
    dist.all_reduce(t, group=pg)
    return pg._get_backend(dev)._comm_ptr()


def run_rccl(backend, addr, meta, tile_offsets, out=None, group=None, stream=None):
    """The whole coherent run of this rank's shards with the exchange in the C
    ABI (gg_coherent_run_ranks: gg_round_exchange over the group's RCCL
    communicator at every quantum boundary) - the same rounds as `run`,
    without a host round trip per collective."""
    backend.coherent_run_ranks(rccl_comm_ptr(group), addr, meta, tile_offsets, out, stream)
