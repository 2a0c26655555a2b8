"""Data parallelism: one process per GPU (torchrun), gradients averaged with one
all-reduce of the optimizer's flat fp32 buffer over RCCL/xGMI ("nccl" backend on
ROCm), or gloo on CPU for the multi-process tests.

The reference is single-device (train.py:55); this is the build's addition
(SURVEY.md §8e): every rank runs the full step on its 64-sample shard, the
decoder gradient (59.6 MB at the reference dims) is averaged, then every rank
applies the identical clamp+Adam update. Initial weights are broadcast from
rank 0. BatchNorm statistics stay per replica (no SyncBN), which equals the
reference at its per-device batch; running statistics are kept per rank.
"""
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistCtx:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = ""

    @property
    def distributed(self):
        """True when collectives run: world > 1, or a one-rank process group forced with
        CAPMI_DIST_FORCE=1 (runs the RCCL path, all-reduce over one rank, on a one-GPU box)."""
        return self.world > 1 or self.backend != ""


def init_from_env(device=None, backend=None):
    """Reads RANK / WORLD_SIZE / LOCAL_RANK (torchrun); MASTER_ADDR defaults to 127.0.0.1.
    CAPMI_DIST_FORCE=1 initialises the process group at world size 1 too (the data-parallel path
    with its collectives on one GPU: how the RCCL branch is exercised without a second device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device is None or (isinstance(device, torch.device) and device.type == "cuda") or device == "cuda":
        device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    device = torch.device(device)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    force = os.environ.get("CAPMI_DIST_FORCE", "0") == "1"
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        be = backend or ("nccl" if device.type == "cuda" else "gloo")
        kw = {"device_id": device} if be == "nccl" else {}
        dist.init_process_group(be, rank=rank, world_size=world, **kw)
    be = dist.get_backend() if dist.is_initialized() else ""
    return DistCtx(rank, world, local, device, be)


def broadcast_module(module, ctx):
    if not ctx.distributed:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, 0)


def allreduce_mean_(buffers, ctx, async_op=False):
    """Average flat gradient buffers across ranks. Returns the work handles if async."""
    if not ctx.distributed:
        return []
    works = []
    for buf in buffers:
        if ctx.backend == "nccl":
            works.append(dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=async_op))
        else:  # gloo has no AVG
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, async_op=False)
            buf.mul_(1.0 / ctx.world)
            works.append(w)
    return [w for w in works if w is not None] if async_op else []


def sampler_for(dataset, ctx):
    if not ctx.distributed:
        return None
    return torch.utils.data.distributed.DistributedSampler(dataset, num_replicas=ctx.world,
                                                           rank=ctx.rank, shuffle=True)


def max_over_ranks(x, ctx):
    """max of a host float over ranks (bench timing)."""
    if not ctx.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=ctx.device if ctx.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_floats(x, ctx):
    """[x of rank 0, x of rank 1, ...] on every rank (bench: per-rank step times)."""
    if not ctx.distributed:
        return [float(x)]
    dev = ctx.device if ctx.backend == "nccl" else "cpu"
    t = torch.zeros(ctx.world, dtype=torch.float64, device=dev)
    t[ctx.rank] = x
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def barrier(ctx):
    if ctx.distributed:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()
