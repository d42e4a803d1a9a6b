"""One-process-per-GPU runtime (replaces Spark's driver/executor bootstrap,
``SparkConf().setAppName("HAR").setMaster(master)`` / ``SparkContext`` at
``Main/main.py:8-9``).

``init()`` reads the ``torch.distributed.run`` environment (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR/PORT), pins the process to ``cuda:LOCAL_RANK`` and
creates the process group: backend ``nccl`` — which IS RCCL on ROCm, running
over xGMI between the GPUs of a node — when GPUs are present, ``gloo``
otherwise (CPU tests exercise the same code path).  Without the env it is a
single-process world of size 1 with no process group at all, unless
``HAR_DIST_FORCE_PG=1``: then a 1-rank group is created anyway (RCCL on a GPU), so
the collective paths — communicator setup, device-buffer reduce-scatter /
all-gather, ``barrier(device_ids)``, host-scalar staging — run on one GPU
(tests/test_gpu_rccl.py; ``DistContext.forced``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    local_rank: int
    world_size: int
    device: torch.device
    backend: Optional[str]
    group: Optional[object] = None
    forced: bool = False  # a 1-rank process group created by HAR_DIST_FORCE_PG=1

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def collective(self) -> bool:
        """True when the DP code paths issue real collectives: world > 1, or a forced 1-rank group."""
        return self.world_size > 1 or self.forced

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init(expected_world: Optional[int] = None, backend: Optional[str] = None, device: Optional[str] = None,
         timeout_s: Optional[int] = None) -> DistContext:
    """``timeout_s`` (default ``HAR_DIST_TIMEOUT_S`` or 600) bounds every collective: a rank that
    stalls or dies makes its peers raise instead of blocking forever, and ``torchrun
    --max-restarts`` then restarts the group from the newest checkpoint."""
    if timeout_s is None:
        timeout_s = int(os.environ.get("HAR_DIST_TIMEOUT_S", "600"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if expected_world is not None and world != expected_world and world > 1:
        raise RuntimeError(f"launched with WORLD_SIZE={world} but --gpus {expected_world}")
    use_cuda = torch.cuda.is_available() and (device is None or str(device).startswith("cuda"))
    # rehearsal of an N-rank job on fewer GPUs (e.g. 8 gloo ranks on one MI355X): HAR_DIST_SHARE_DEVICE=1
    # puts every rank on cuda:0, HAR_DIST_BACKEND picks the backend (gloo: host-staged collectives)
    share = os.environ.get("HAR_DIST_SHARE_DEVICE", "0") == "1"
    backend = backend or os.environ.get("HAR_DIST_BACKEND") or None
    if use_cuda:
        dev_index = 0 if share else local_rank
        torch.cuda.set_device(dev_index)
        dev = torch.device("cuda", dev_index)
    else:
        dev = torch.device("cpu")
    be = None
    forced = world == 1 and os.environ.get("HAR_DIST_FORCE_PG", "0") == "1"
    if world > 1 or forced:
        be = backend or ("nccl" if use_cuda else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if forced and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if restart > 0 and not dist.is_initialized():
            # under torchrun --max-restarts the rendezvous store can outlive a failed attempt: key
            # this attempt's process group under its own prefix, or a restarted rank may read a dead
            # peer's (stale) transport address from the previous attempt and fail to connect
            store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world,
                                               timeout=datetime.timedelta(seconds=timeout_s)))
            kw["store"] = dist.PrefixStore(f"har/attempt{restart}", store)
        if not dist.is_initialized():
            dist.init_process_group(**kw)
    return DistContext(rank, local_rank, world, dev, be, None, forced)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def barrier(ctx: DistContext):
    if ctx.collective:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier(group=ctx.group)


def sync(device):
    if isinstance(device, torch.device) and device.type == "cuda":
        torch.cuda.synchronize(device)


def _reduce_scalar(ctx: DistContext, x: float, op) -> float:
    if not ctx.collective:
        return x
    from . import comm

    t = torch.tensor([x], dtype=torch.float64)
    comm.all_reduce(t, op=op, group=ctx.group)  # (staged to the device under RCCL)
    return float(t.item())


def max_over_ranks(ctx: DistContext, x: float) -> float:
    return _reduce_scalar(ctx, x, dist.ReduceOp.MAX)


def sum_over_ranks(ctx: DistContext, x: float) -> float:
    return _reduce_scalar(ctx, x, dist.ReduceOp.SUM)


def mean_over_ranks(ctx: DistContext, x: float) -> float:
    return sum_over_ranks(ctx, x) / ctx.world_size


def shutdown(ctx: DistContext):
    if ctx.collective and dist.is_initialized():
        barrier(ctx)
        dist.destroy_process_group()


def shard_range(n: int, rank: int, world: int):
    """Contiguous [lo, hi) row range of ``rank`` (global row ids stay meaningful)."""
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return lo, hi
