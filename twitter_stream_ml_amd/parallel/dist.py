"""Process-group bootstrap and collectives (one process per GPU).

Control plane: ``torch.distributed`` (``nccl`` = RCCL on ROCm for GPU jobs,
``gloo`` for the CPU engine), initialised from the usual ``RANK`` /
``WORLD_SIZE`` / ``LOCAL_RANK`` / ``MASTER_ADDR`` / ``MASTER_PORT`` variables
that ``torch.distributed.run`` sets.

Data plane on GPUs: the engine's own RCCL communicator (``csrc/hip/comm.cpp``)
issues the per-iteration gradient all-reduce on the engine's compute stream
with no Python in the loop.  Its ``ncclUniqueId`` is created on rank 0 and
broadcast here.  This replaces Spark's broadcast + treeAggregate per GD
iteration.

The CPU engine gets :func:`allreduce_fn`, a numpy float64 sum over gloo —
the same call sites, so DP on CPU and on GPUs run identical algorithms.
"""
from __future__ import annotations

import datetime
import os
import sys
import threading
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

__all__ = ["DistInfo", "init_distributed", "dist_info", "make_rccl_comm", "make_comm", "broadcast_flag",
           "allreduce_fn",
           "barrier", "allreduce_max_scalar", "allreduce_sum_scalar", "allreduce_min_scalar", "shutdown",
           "check_replicas", "replica_digest", "replicas_identical", "ReplicaDivergence", "gather_to_main",
           "gather_parts"]


@dataclass(frozen=True)
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


_INFO = DistInfo()


def dist_info() -> DistInfo:
    return _INFO


def init_distributed(backend: Optional[str] = None, device: Optional[int] = None,
                     timeout_s: float = 600.0) -> DistInfo:
    """Initialise the default process group if ``WORLD_SIZE > 1``."""
    global _INFO
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        _INFO = DistInfo(0, 1, local, "none")
        return _INFO
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kwargs = {}
    if backend == "nccl":
        dev = local if device is None else device
        torch.cuda.set_device(dev)
        kwargs["device_id"] = torch.device("cuda", dev)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    _INFO = DistInfo(rank, world, local, backend)
    return _INFO


def make_rccl_comm(device: int, force: bool = False):
    """Engine-owned RCCL communicator for this process (None when world == 1,
    unless ``force``: a world-1 communicator, so an engine built with
    ``force_dp`` runs its whole DP path -- every collective -- through RCCL
    on one GPU)."""
    info = dist_info()
    if info.world <= 1:
        if not force:
            return None
        from ..ops._native import hip
        h = hip()
        return h.Comm(h.rccl_unique_id(), 0, 1, int(device))
    import torch.distributed as dist
    from ..ops._native import hip
    h = hip()
    obj = [h.rccl_unique_id() if info.rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return h.Comm(obj[0], info.rank, info.world, int(device))


def make_comm(device: int, kind: str = "rccl", own_group: bool = False, force: bool = False):
    """Engine communicator: ``rccl`` (device collectives on the engine stream,
    one GPU per rank) or ``gloo`` (host-staged through torch.distributed
    gloo, so N ranks may share one GPU: the real multi-process engine path,
    testable on a single MI355X).  None when world == 1 unless ``force``
    (a world-1 RCCL communicator for forced-DP engines).  ``own_group``:
    gloo collectives on a process group of their own (a second communicator
    used concurrently with the first, e.g. the engine's prep communicator;
    every RCCL communicator is its own)."""
    info = dist_info()
    if info.world <= 1 and not (force and kind == "rccl"):
        return None
    if kind == "rccl":
        return make_rccl_comm(device, force=force)
    if kind != "gloo":
        raise ValueError(f"unknown comm {kind!r}")
    import torch
    import torch.distributed as dist
    from ..ops._native import hip
    group = None if (info.backend == "gloo" and not own_group) else dist.new_group(backend="gloo")
    ops = {0: dist.ReduceOp.SUM, 1: dist.ReduceOp.MAX, 2: dist.ReduceOp.MIN}
    # unsigned buffers reduce as their signed twins (sums wrap identically);
    # MAX / MIN only ever see u8 flags, which torch / gloo handle natively
    as_signed = {np.dtype("u4"): np.dtype("i4"), np.dtype("u8"): np.dtype("i8")}

    trace = os.environ.get("TWTML_COMM_TRACE")
    label = "prep" if own_group else "main"

    def collective(arr: np.ndarray, op: int, root: int) -> None:
        if trace:   # debugging collective order across ranks / threads
            print(f"[comm r{info.rank} {label} {threading.get_ident() % 100000}] op {op} n {arr.size} "
                  f"{arr.dtype}", file=sys.stderr, flush=True)
        a = arr.view(as_signed.get(arr.dtype, arr.dtype))
        t = torch.from_numpy(a)
        if op == -1:
            dist.broadcast(t, src=root, group=group)
        elif op == -2:
            parts = list(t.chunk(info.world))
            mine = parts[info.rank].clone()
            dist.all_gather(parts, mine, group=group)
        else:
            dist.all_reduce(t, op=ops[op], group=group)

    return hip().HostComm(info.rank, info.world, collective)


def allreduce_fn() -> Optional[Callable[[np.ndarray], np.ndarray]]:
    """float64 sum across ranks (gloo/nccl via torch), or None for 1 rank."""
    info = dist_info()
    if info.world <= 1:
        return None
    import torch
    import torch.distributed as dist

    def _allreduce(v: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64).copy())
        if info.backend == "nccl":
            t = t.cuda()
        if info.world <= 2:   # a + b == b + a: every rank gets the same bits
            dist.all_reduce(t)
            return t.cpu().numpy()
        # > 2 ranks: gloo's summation order differs between ranks; all-gather
        # and add in rank order so the replicas stay bit-identical
        parts = [torch.empty_like(t) for _ in range(info.world)]
        dist.all_gather(parts, t)
        acc = parts[0].cpu().numpy().copy()
        for p in parts[1:]:
            acc += p.cpu().numpy()
        return acc

    return _allreduce


def barrier() -> None:
    info = dist_info()
    if info.world > 1:
        import torch.distributed as dist
        dist.barrier()


def _reduce_scalar(x: float, op: str) -> float:
    info = dist_info()
    if info.world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64)
    if info.backend == "nccl":
        t = t.cuda()
    red = {"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}.get(op, dist.ReduceOp.SUM)
    dist.all_reduce(t, op=red)
    return float(t.item())


def allreduce_max_scalar(x: float) -> float:
    return _reduce_scalar(x, "max")


def allreduce_sum_scalar(x: float) -> float:
    return _reduce_scalar(x, "sum")


def allreduce_min_scalar(x: float) -> float:
    return _reduce_scalar(x, "min")


class ReplicaDivergence(RuntimeError):
    """Data-parallel replicas of the model no longer agree bit for bit."""


def replica_digest(arr: np.ndarray) -> int:
    """64-bit digest of an array's bytes (order-sensitive, exact)."""
    import hashlib
    h = hashlib.blake2b(np.ascontiguousarray(arr).tobytes(), digest_size=8)
    return int.from_bytes(h.digest(), "little", signed=True)


def check_replicas(arr: np.ndarray, what: str = "model") -> None:
    """Race/divergence detector: all ranks must hold identical
    replicas.  MIN and MAX all-reduces of a digest differ iff any rank
    disagrees; raises :class:`ReplicaDivergence` on every rank."""
    info = dist_info()
    if info.world <= 1:
        return
    import torch
    import torch.distributed as dist
    d = replica_digest(arr)
    dev = "cuda" if info.backend == "nccl" else "cpu"
    lo = torch.tensor([d], dtype=torch.int64, device=dev)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if int(lo.item()) != int(hi.item()):
        raise ReplicaDivergence(f"{what} replicas diverged across ranks (digest on rank "
                                f"{info.rank}: {d:#x})")


def replicas_identical(arr: np.ndarray) -> bool:
    """:func:`check_replicas` as a verdict instead of an exception: True when
    every rank's replica has the same digest (True at world 1)."""
    try:
        check_replicas(arr)
    except ReplicaDivergence:
        return False
    return True


def broadcast_flag(flag: bool) -> bool:
    """Rank 0's boolean on every rank (True/False as the max of 0/1 with the
    other ranks contributing 0)."""
    if dist_info().world <= 1:
        return bool(flag)
    v = 1.0 if (flag and dist_info().rank == 0) else 0.0
    return _reduce_scalar(v, "max") > 0.5


def gather_to_main(arr: np.ndarray, group=None) -> Optional[np.ndarray]:
    """Concatenate every rank's 1-D float64 array on rank 0 (None elsewhere).

    CS7/CS11: the reference ``collect``s the batch's real/predicted values to
    the driver for the Lightning plot; here each rank's sample is gathered
    once per batch by the plot shipper thread (``report/plot_shipper.py``) on
    a gloo ``group`` of its own, off the training path."""
    parts = gather_parts(arr, group)
    return None if parts is None else np.concatenate(parts)


def gather_parts(arr: np.ndarray, group=None) -> Optional[list]:
    """Every rank's 1-D float64 array on rank 0, one entry per rank in rank
    order (None elsewhere)."""
    info = dist_info()
    a = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)
    if info.world <= 1:
        return [a]
    import torch
    import torch.distributed as dist
    dev = "cuda" if (info.backend == "nccl" and group is None) else "cpu"
    n = torch.tensor([a.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(info.world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes) if sizes else 0
    buf = torch.zeros(max(m, 1), dtype=torch.float64, device=dev)
    buf[:a.shape[0]] = torch.from_numpy(a).to(dev)
    parts = [torch.zeros_like(buf) for _ in range(info.world)]
    dist.all_gather(parts, buf, group=group)   # all_gather: supported by gloo and RCCL alike
    if info.rank != 0:
        return None
    return [p[:s].cpu().numpy() for p, s in zip(parts, sizes)]


def shutdown() -> None:
    info = dist_info()
    if info.world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
