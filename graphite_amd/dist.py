"""Multi-GPU plumbing: one process per GPU (torchrun), tiles sharded by rank.

The reference spreads tiles over processes (Config process map,
common/misc/config.cc:199-228) and exchanges coherence traffic over its TCP
transport.  In private-cache mode the (tile, L1-D set) units are independent,
so ranks simulate disjoint tile ranges with NO data-path collective; the only
collectives are the barrier / max-reduction of the timing and the final
gather of per-tile counters (torch.distributed: RCCL on GPUs, gloo on CPU).
"""
import os

import numpy as np


def env():
    """(world, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def tile_range(rank, tiles_per_rank):
    """Global tile ids simulated by `rank` (weak scaling: fixed tiles per rank)."""
    return rank * tiles_per_rank, (rank + 1) * tiles_per_rank


def init(backend="nccl"):
    import torch.distributed as dist
    world, _, _ = env()
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend)
    return world > 1


def _device(backend):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def barrier():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def max_over_ranks(x, backend="nccl"):
    """Max of a float over ranks (the slowest rank defines the step time)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_device(backend))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_tile_counters(local, rank, world, backend="nccl"):
    """Per-tile counters of every rank, indexed by global tile id
    ([world * T, ...] uint64); identical on all ranks."""
    import torch
    import torch.distributed as dist
    local = np.ascontiguousarray(local, np.uint64)
    T = local.shape[0]
    full = np.zeros((world * T,) + local.shape[1:], np.uint64)
    full[rank * T:(rank + 1) * T] = local
    if not (dist.is_available() and dist.is_initialized()) or world == 1:
        return full
    t = torch.from_numpy(full.view(np.int64)).to(_device(backend))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().view(np.uint64)
