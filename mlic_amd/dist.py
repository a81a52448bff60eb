"""Image-sharded multi-GPU execution.

Images are independent: one process per GPU, jobs assigned by longest-processing-time-first on
their padded pixel count (a 4K image weighs ~4x a 1080p one), no cross-GPU context.  The only
collective is an all_gather of fixed-size per-image records after the work — the role of
`dist.gather_object` in playground/compression_trainer.py:857-858 — over RCCL ("nccl" backend on
ROCm, xGMI) or gloo (CPU tests).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

# per-image record layout (float64): job id, H, W, level, bytes, bpp_file, bpp_lik, mse, psnr,
# enc_ms, dec_ms
RECORD_FIELDS = ("job", "H", "W", "level", "bytes", "bpp_file", "bpp_lik", "mse", "psnr", "enc_ms", "dec_ms")
RECORD_LEN = len(RECORD_FIELDS)


def padded_pixels(h: int, w: int) -> int:
    return ((h + 63) // 64 * 64) * ((w + 63) // 64 * 64)


def lpt_shard(sizes: Sequence[Tuple[int, int]], world: int) -> List[List[int]]:
    """Greedy LPT: jobs sorted by padded pixel count (descending) to the least-loaded rank.
    Deterministic (ties broken by job index, then rank)."""
    order = sorted(range(len(sizes)), key=lambda i: (-padded_pixels(*sizes[i]), i))
    heap = [(0, r) for r in range(world)]
    heapq.heapify(heap)
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + padded_pixels(*sizes[i]), r))
    for r in out:
        r.sort()
    return out


def group_shard(keys: Sequence, sizes: Sequence[Tuple[int, int]], world: int) -> List[List[int]]:
    """Contiguous partition of the jobs, ordered by their batch key (weight set, shape), into `world`
    slices of near-equal padded pixel count (each within one job's weight of its share).  A rank then
    runs a few whole batches instead of the one or two images of every (weights, shape) group that
    LPT deals it round-robin (BASELINE config 4: 144 equal jobs in 12 groups -> 18 jobs in <= 3
    batches per rank at world 8).  Deterministic."""
    order = sorted(range(len(keys)), key=lambda i: (keys[i], i))
    w = [padded_pixels(*sizes[i]) for i in order]
    total = float(sum(w))
    out: List[List[int]] = [[] for _ in range(world)]
    acc, r = 0.0, 0
    for i, wi in zip(order, w):
        while r < world - 1 and acc + 0.5 * wi > total * (r + 1) / world:
            r += 1
        out[r].append(i)
        acc += wi
    for s in out:
        s.sort()
    return out


def gather_records(local: torch.Tensor, max_per_rank: int) -> torch.Tensor:
    """all_gather fixed-size [max_per_rank, RECORD_LEN] float64 blocks (rows with job = -1 are
    padding) and return the valid rows sorted by job id.  Works single-process too."""
    assert local.dim() == 2 and local.shape[1] == RECORD_LEN and local.shape[0] <= max_per_rank
    dev = local.device
    block = torch.full((max_per_rank, RECORD_LEN), -1.0, dtype=torch.float64, device=dev)
    block[: local.shape[0]] = local.to(torch.float64)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        parts = [torch.empty_like(block) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, block)
        block = torch.cat(parts)
    rows = block[block[:, 0] >= 0]
    return rows[torch.argsort(rows[:, 0])]
