"""Process-group bootstrap: one process per GPU, RCCL over xGMI (``backend="nccl"`` is RCCL on
ROCm), gloo on CPU for tests.

The reference has no collectives at all: its only cross-worker mechanism is
Redis.  Here multi-GPU serving is ``torchrun --nproc-per-node N``: each rank owns the rooms
``r ≡ rank (mod N)`` (``parallel.rooms``), and the control/data plane uses a handful of small,
latency-bound collectives (broadcast of round secrets, all-gather of images/scores, barrier at
round boundaries).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Any, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: Optional[str]

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _inject_init_fault(rank: int) -> None:
    """Test hook (SURVEY §5.3 fault injection): ``CASSMANTLE_FAULT_DIST_INIT=raise|hang`` makes
    the ranks listed in ``CASSMANTLE_FAULT_DIST_RANKS`` (comma-separated, default every rank)
    fail or wedge at the process-group init, as a broken RCCL / xGMI setup would."""
    mode = os.environ.get("CASSMANTLE_FAULT_DIST_INIT")
    if not mode:
        return
    ranks = os.environ.get("CASSMANTLE_FAULT_DIST_RANKS")
    if ranks and str(rank) not in ranks.split(","):
        return
    if mode == "raise":
        raise RuntimeError(f"injected process-group init failure on rank {rank} (CASSMANTLE_FAULT_DIST_INIT)")
    if mode == "hang":
        import time
        time.sleep(1e6)


def init_from_env(backend: Optional[str] = None, timeout_s: float = 600.0) -> DistContext:
    """Reads RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT (torchrun contract)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    be = None
    _inject_init_fault(rank)
    if world > 1:
        # CASSMANTLE_DIST_BACKEND=gloo: rehearse the multi-rank path with several ranks on ONE GPU
        # (RCCL refuses two ranks on a device); production is always nccl (= RCCL) on GPUs
        be = backend or os.environ.get("CASSMANTLE_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        if not dist.is_initialized():
            dist.init_process_group(**kw)
    return DistContext(rank, world, local, device, be)


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        try:
            dist.barrier()
        except Exception:  # noqa: BLE001
            pass
        dist.destroy_process_group()


def broadcast_object(obj: Any, src: int = 0, group=None) -> Any:
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]


def all_gather_object(obj: Any) -> List[Any]:
    if not (dist.is_available() and dist.is_initialized()):
        return [obj]
    out: List[Any] = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
