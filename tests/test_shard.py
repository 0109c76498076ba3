"""Multi-GPU sharding logic on CPU: LPT plan properties and the one counter
collective, exercised with world_size-2 gloo process groups."""
import os
import socket

import pytest

from photohive_dsp_amd import shard


def test_assign_partitions_every_image_once():
    sizes = shard.mixed_sizes(4096, 7)
    for world in (1, 2, 4, 8):
        plan = shard.assign(sizes, world)
        flat = sorted(i for r in plan for i in r)
        assert flat == list(range(len(sizes)))
        ld = shard.loads(sizes, plan)
        # LPT bound: max load <= mean + largest item
        biggest = max(h * w for h, w in sizes)
        assert max(ld) <= sum(ld) / world + biggest


def test_assign_is_deterministic_and_balanced():
    sizes = shard.mixed_sizes(4096, 3)
    a, b = shard.assign(sizes, 8), shard.assign(list(sizes), 8)
    assert a == b
    ld = shard.loads(sizes, a)
    assert max(ld) / min(ld) < 1.01          # 4096 images: near-perfect balance


def test_assign_uniform_sizes_round_robin_counts():
    sizes = [(3000, 4000)] * 2048            # config 4: 256 per GPU
    plan = shard.assign(sizes, 8)
    assert [len(p) for p in plan] == [256] * 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sizes = shard.mixed_sizes(257, 11)
        plan = shard.assign(sizes, world)
        mine = plan[rank]
        pix = sum(sizes[i][0] * sizes[i][1] for i in mine)
        m = shard.merge_counters([0.5 + rank, float(len(mine)), float(pix), 3.0 * pix])
        el, n, p = m["elapsed"], m["images"], m["pixels"]
        assert m["alg_bytes"] == 3.0 * sum(h * w for h, w in sizes)
        assert m["per_rank_elapsed"] == [0.5 + r for r in range(world)]
        assert m["ranks"] == world and m["devices"] == world          # no device slots: one per rank
        # a rehearsal with every rank on one card counts ONE device (bench.py's n_gpus)
        one = shard.merge_counters([1.0, 1.0], dev_index=shard.device_of(rank, 1))
        assert (one["ranks"], one["devices"]) == (world, 1), one
        own = shard.merge_counters([1.0, 1.0], dev_index=shard.device_of(rank, 8))
        assert (own["ranks"], own["devices"]) == (world, world), own
        got = [None] * world
        dist.all_gather_object(got, mine)
        q.put((rank, el, n, p, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_counter_merge_and_disjoint_shards(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = shard.mixed_sizes(257, 11)
    total_pix = sum(h * w for h, w in sizes)
    for rank, el, n, p, got in res:
        assert el == 0.5 + (world - 1)       # max over ranks
        assert n == 257 and p == total_pix   # sums over ranks
        flat = sorted(i for r in got for i in r)
        assert flat == list(range(257))
