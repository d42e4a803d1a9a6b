"""Backend-aware collectives: every DP call site of the package goes through these.

The production path is RCCL (backend ``nccl`` on ROCm) over xGMI with HBM-resident tensors:
the tensors go straight to ``torch.distributed`` and nothing is staged.  Two other placements
occur and are handled here, once, instead of at every call site:

* gloo with device tensors — the rehearsal of an N-rank job on one MI355X
  (``HAR_DIST_SHARE_DEVICE=1``: N gloo ranks share ``cuda:0``; tests/test_gpu_dp.py): gloo
  reduces host buffers, so the tensor is staged through the host and copied back;
* RCCL with host tensors (a host-side count or size): staged through the rank's device.

The reference has no explicit collectives at all — every combine is inside Spark
(``treeAggregate`` / ``reduceByKey`` / ``collect``).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


def backend(group=None) -> str:
    return str(dist.get_backend(group)).lower()


def _home(t: torch.Tensor, be: str) -> torch.device:
    """Where the backend wants the buffer: host for gloo, the current device for RCCL."""
    if be == "gloo":
        return torch.device("cpu")
    if be == "nccl":
        return t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
    return t.device


def _staged(t: torch.Tensor, be: str) -> torch.Tensor:
    home = _home(t, be)
    if t.device == home and t.is_contiguous():
        return t
    return t.to(home).contiguous()


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce of ``t`` (any placement)."""
    be = backend(group)
    s = _staged(t, be)
    dist.all_reduce(s, op=op, group=group)
    if s is not t:
        t.copy_(s)
    return t


def all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group=None) -> torch.Tensor:
    be = backend(group)
    so, si = _staged(out, be), _staged(inp, be)
    dist.all_gather_into_tensor(so, si, group=group)
    if so is not out:
        out.copy_(so)
    return out


def reduce_scatter_tensor(out: torch.Tensor, inp: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    be = backend(group)
    so, si = _staged(out, be), _staged(inp, be)
    dist.reduce_scatter_tensor(so, si, op=op, group=group)
    if so is not out:
        out.copy_(so)
    return out


def broadcast(t: torch.Tensor, src: int, group=None) -> torch.Tensor:
    be = backend(group)
    s = _staged(t, be)
    dist.broadcast(s, src=src, group=group)
    if s is not t:
        t.copy_(s)
    return t


def send_recv(sends: List[tuple], recvs: List[tuple], group=None) -> None:
    """Point-to-point exchange: ``sends`` [(tensor, dst)], ``recvs`` [(tensor, src)] posted as one
    batch (``batch_isend_irecv``), every receive copied back to its tensor after the waits."""
    be = backend(group)
    ops, back = [], []
    for t, peer in sends:
        ops.append(dist.P2POp(dist.isend, _staged(t, be), peer, group=group))
    for t, peer in recvs:
        s = _staged(t, be)
        ops.append(dist.P2POp(dist.irecv, s, peer, group=group))
        if s is not t:
            back.append((t, s))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    for t, s in back:
        t.copy_(s)


def world_of(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def rank_of(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def barrier(group=None, device: Optional[torch.device] = None) -> None:
    if backend(group) == "nccl" and device is not None and device.type == "cuda":
        dist.barrier(group=group, device_ids=[device.index])
    else:
        dist.barrier(group=group)
