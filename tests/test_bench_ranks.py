"""bench.py's multi-rank path on the CPU: `python bench.py --gpus 2` with no
torchrun environment starts the ranks itself (a torch.distributed.run child),
every rank takes its shard of configs 2, 4 and 5 and one gloo all-gather
merges the counters; rank 0 prints one JSON line with both ranks' images."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_spawns_ranks_and_merges_counters():
    env = dict(os.environ, PHD_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plan-only",
                        "--batch", "8", "--config4-images", "64", "--config5-images", "96"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["config2"]["images"] == 2 * 8                      # weak: batch 8 per rank
    assert d["config4"]["images"] == 64 and d["config5"]["images"] == 96   # strong: totals split
    from photohive_dsp_amd import shard
    sizes = shard.mixed_sizes(96, 5)
    assert d["config5"]["pixels"] == sum(h * w for h, w in sizes)
    assert d["config2"]["elapsed_max"] == 2.0                   # max over ranks (1 + rank)
