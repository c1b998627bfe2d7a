"""CU-masked HIP streams: reserve a few compute units for latency-critical work.

BASELINE config 5 overlaps image generation with streaming guess scoring on one GPU.  A
high-priority stream only lets the scorer's kernels be *dispatched* first; once the denoise
loop's workgroups occupy every CU (a captured UNet step is ~360 kernels of up to ~460 us), a
scoring kernel still waits for CUs to drain.  Here the scorer owns ``reserve`` CUs through a
stream created with ``hipExtStreamCreateWithCUMask`` and the generation stream gets the
complement, so neither ever waits on the other's workgroups (verdict r2 item 6; reference: the
score request is served inline on the request path, ``/root/reference/main.py:113-120``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch


def split_cus(total: int, reserve: int) -> Tuple[List[int], List[int]]:
    """(reserved, rest): ``reserve`` CUs spread evenly over the id range (the CUs of one XCD are
    contiguous ids, so this spreads the reservation over the XCDs and their L2s)."""
    reserve = max(0, min(reserve, total - 1))
    if reserve == 0:
        return [], list(range(total))
    step = total / reserve
    mine = sorted({int(i * step) for i in range(reserve)})
    rest = [c for c in range(total) if c not in set(mine)]
    return mine, rest


def mask_words(cus: Sequence[int], total: int) -> List[int]:
    words = [0] * ((total + 31) // 32)
    for c in cus:
        words[c // 32] |= 1 << (c % 32)
    return words


def masked_stream(device, cus: Sequence[int]) -> "torch.cuda.ExternalStream":
    from ..ops._ext import ext
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    total = int(ext().cu_count(idx))
    handle = ext().cu_mask_stream(idx, mask_words(cus, total))
    return torch.cuda.ExternalStream(handle, device=torch.device("cuda", idx))


def reserved_streams(device, reserve: int) -> Tuple[Optional["torch.cuda.ExternalStream"],
                                                    Optional["torch.cuda.ExternalStream"]]:
    """(scorer stream on ``reserve`` CUs, generation stream on the rest), or (None, None)."""
    if reserve <= 0 or torch.device(device).type != "cuda":
        return None, None
    from ..ops._ext import ext
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    total = int(ext().cu_count(idx))
    mine, rest = split_cus(total, reserve)
    return masked_stream(device, mine), masked_stream(device, rest)
