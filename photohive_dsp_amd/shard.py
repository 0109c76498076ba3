"""Multi-GPU sharding of independent images.

Images are independent and each fits one GPU, so the batch is partitioned
across ranks with no data-path collective: every rank reports on its own
images and keeps its results.  The only collective merges a few counters
(images, pixels, wall time) -- one all-reduce SUM whose wall-time slots are
one-hot per rank, so the max is taken after it -- over RCCL (backend "nccl")
on the GPU box or gloo in the CPU tests.

Mixed sizes (BASELINE.json config 5) are balanced with a static LPT
assignment: images sorted by pixel count, largest first, each onto the
least-loaded rank (ties: lower rank, then lower index -- deterministic, so
every rank computes the same plan without communicating).
"""
from __future__ import annotations

import heapq
from typing import List, Sequence, Tuple

# config 5's size list (2*3*5-smooth shapes, aspect within 1:5..5:1), SURVEY.md 8d
MIXED_SHAPES = [(512, 512), (480, 640), (720, 1280), (1080, 1920), (1536, 2048), (2000, 3000),
                (3000, 4000), (4000, 6000), (640, 480), (1280, 720), (3000, 2000), (6000, 4000)]


def mixed_sizes(n: int, seed: int) -> List[Tuple[int, int]]:
    """n (H, W) shapes drawn by seed from MIXED_SHAPES (splitmix64, as synth)."""
    from .synth import splitmix64
    words = splitmix64(seed, n)
    return [MIXED_SHAPES[int(w % len(MIXED_SHAPES))] for w in words]


def assign(sizes: Sequence[Tuple[int, int]], world: int) -> List[List[int]]:
    """LPT partition of image indices over `world` ranks by pixel count.
    Returns per-rank index lists, each in ascending image order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i][0] * sizes[i][1], i))
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + sizes[i][0] * sizes[i][1], r))
    return [sorted(x) for x in out]


def loads(sizes: Sequence[Tuple[int, int]], plan: List[List[int]]) -> List[int]:
    """Pixels per rank of a plan."""
    return [sum(sizes[i][0] * sizes[i][1] for i in idx) for idx in plan]


COUNTERS = ("elapsed", "images", "pixels", "alg_bytes", "kernel_ms", "launches")
MAX_DEVICES = 64          # device-index slots per node (one-hot, like the wall times)


def device_of(local_rank: int, visible: int) -> int:
    """The device a rank drives: LOCAL_RANK modulo the visible devices (a
    rehearsal with more ranks than cards puts several ranks on one card; with
    no device visible, the rank's own index -- the plan of a real node)."""
    return local_rank % visible if visible > 0 else local_rank


def merge_counters(values, device=None, dev_index=None):
    """The single collective: ONE all-reduce (SUM) over the
    default process group (RCCL over xGMI on the GPU box, gloo in the CPU
    tests; identity when torch.distributed is not initialised) of this rank's
    counter vector {elapsed s, images, pixels, algorithmic bytes, kernel ms,
    kernel launches} followed by a one-hot row of world slots holding its wall
    time at its rank and, when dev_index is given, a one-hot row of device
    slots.  Every rank gets the merge: the sums of the counters, the max of
    the wall times (from the one-hot slots), each rank's wall time
    (per_rank_elapsed), the ranks and the number of DISTINCT devices they ran
    on (`devices`: a two-rank rehearsal on one card is 2 ranks, 1 device)."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in values] + [0.0] * (len(COUNTERS) - len(values))
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    world, rank = (dist.get_world_size(), dist.get_rank()) if multi else (1, 0)
    slots = [0.0] * world
    slots[rank] = vals[0]
    devs = [0.0] * MAX_DEVICES
    if dev_index is not None:
        if not 0 <= dev_index < MAX_DEVICES:
            raise ValueError(f"device index {dev_index} outside [0, {MAX_DEVICES})")
        devs[dev_index] = 1.0
    t = torch.tensor(vals + slots + devs, dtype=torch.float64, device=device)
    if multi:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    row = t.cpu().tolist()
    res = {k: row[j] for j, k in enumerate(COUNTERS)}
    per_rank = row[len(COUNTERS):len(COUNTERS) + world]
    res["elapsed"] = max(per_rank)
    res["per_rank_elapsed"] = per_rank
    res["ranks"] = world
    res["devices"] = sum(1 for x in row[len(COUNTERS) + world:] if x > 0) if dev_index is not None else world
    return res
