"""Benchmark: images/s of the full PhotoHive_DSP report on 4000x3000 RGB8 images
(BASELINE.json config 2 at N=1; weak-scaled batches per GPU for N>1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A step = one full report (stats, S-bar, palette, blur profile, blur vectors)
of every image of one device-resident batch of B images per GPU.  Images are
synthetic (splitmix64 uniform RGB8, generated on the device; seed = global
image index).  Ranks shard images with no data-path collective; one small
all-reduce merges the counters.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=8, help="images per GPU per step")
    p.add_argument("--height", type=int, default=3000)
    p.add_argument("--width", type=int, default=4000)
    p.add_argument("--cpu-images", type=int, default=3, help="CPU baseline sample size (images)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="do not bracket kernels with HIP events (roofline then null)")
    p.add_argument("--no-config3", action="store_true",
                   help="skip the BASELINE config-3/4 objects (512 x 1080p statistics pass; FFT + blur path)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                   help="per-kernel PMC traffic summary written by tools/pmc_collect.py")
    return p.parse_args(argv)


def cpu_baseline(h, w, n_images):
    """The C restatement of the reference path (oracle/, -O2) + scipy rfft2 (1 worker),
    one thread, on a bounded sample of the same workload (n_images uniform images)."""
    from oracle import oracle as orc
    from photohive_dsp_amd import synth
    imgs = [synth.uniform(h, w, 10_000 + i) for i in range(n_images)]
    orc.report(synth.uniform(400, 400, 1))        # load the library outside the timing
    t0 = time.perf_counter()
    for im in imgs:
        orc.report(im, fft_workers=1)
    dt = time.perf_counter() - t0
    return {"value": n_images / dt, "unit": "images/s", "cores": 1, "kind": "port",
            "sample": f"{n_images} x {h}x{w} uniform RGB8 full reports, oracle/phd_oracle.c -O2 "
                      f"+ scipy.fft.rfft2 (1 worker), {dt:.1f} s"}


def single_image(lib, last_error, h=3000, w=4000, iters=20):
    """BASELINE config 2 as literally stated: ONE 4000x3000 image per call.
    Median latency of a full report from a device-resident image
    (phd_report_batch_device, batch 1) and from a host buffer
    (phd_report_u8: one 36 MB H2D copy included)."""
    import numpy as np
    import torch
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    nb = h * w * 3
    t = torch.empty(nb, dtype=torch.uint8, device="cuda")
    assert lib.phd_fill_uniform_device(t.data_ptr(), nb, 77, None) == 0, last_error()
    host = t.cpu().numpy()
    cfg = make_config()
    out = (ctypes.POINTER(Full_Report_Data) * 1)()
    st = (ctypes.c_int * 1)()

    def dev():
        if lib.phd_report_batch_device(t.data_ptr(), 1, h, w, nb, ctypes.byref(cfg), out, st, None) != 0:
            raise RuntimeError(last_error())
        r = out[0]
        lib.free_full_report(ctypes.byref(r))

    def hst():
        r = lib.phd_report_u8(host.ctypes.data, h, w, 0, ctypes.byref(cfg), None)
        if not r:
            raise RuntimeError(last_error())
        lib.free_full_report(ctypes.byref(r))

    res = {}
    for name, fn in (("device_resident", dev), ("host_buffer", hst)):
        fn()
        ts = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        res[name + "_ms"] = round(1000 * float(np.median(ts)), 3)
    del t
    torch.cuda.empty_cache()
    return {"workload": f"1 x {h}x{w} RGB8 per call, full report, median of {iters}", **res}


def config3(lib, last_error, n=512, h=1080, w=1920, iters=10):
    """BASELINE config 3 (the HBM-roofline run): the rgb2hsv + rgb_statistics pass
    (phd_hsv_stats_batch_device, stats.hip) over n device-resident 1080p images, one
    launch per batch.  Kernel time from HIP events on the launch stream; algorithmic
    bytes = 3 per pixel."""
    import torch
    from photohive_dsp_amd.structures import RGB_Statistics
    nb = h * w * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, i, None) == 0, last_error()
    st = (RGB_Statistics * n)()
    sat = (ctypes.c_double * n)()

    def run():
        if lib.phd_hsv_stats_batch_device(t.data_ptr(), n, h, w, 0, st, sat, None) != 0:
            raise RuntimeError(f"hsv_stats batch failed: {last_error()}")
    run()
    lib.phd_profile_kernels(0)
    lib.phd_profile_kernels(1)                      # K1 slot = the statistics pass
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    wall = (time.perf_counter() - t0) / iters
    tot, cnt = ctypes.c_double(), ctypes.c_long()
    lib.phd_profile_read(0, ctypes.byref(tot), ctypes.byref(cnt))
    lib.phd_profile_kernels(0)
    us = 1000 * tot.value / max(cnt.value, 1)
    ab = 3.0 * n * h * w
    del t
    torch.cuda.empty_cache()
    return {"workload": f"{n} x {h}x{w} RGB8, rgb2hsv + rgb_statistics only, device-resident",
            "images_per_s": round(n / wall, 1), "ms_per_batch_wall": round(1000 * wall, 3),
            "roofline": {"kernel": "rgb_stats", "bound": "hbm", "achieved": round(ab / (us * 1e-6) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ab / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": ab, "avg_launch_us": round(us, 2)}}


def config4(lib, last_error, n=32, h=3000, w=4000, iters=8):
    """BASELINE config 4 on one GPU: the FFT + blur-profile path alone
    (phd_blur_batch_device) over n device-resident 4000x3000 images.  The
    column pass is this path's dominant kernel: its algorithmic bytes are the
    half spectrum read plus the bin map, 18 * H * (W/2+1) per image (SURVEY.md 8d
    counts 3N + 32 H Wf = 228 MB for the whole path)."""
    import numpy as np
    import torch
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Blur_Vector
    nb = h * w * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, 1000 + i, None) == 0, last_error()
    cfg = make_config()
    bins = np.zeros((n, cfg.angle_partitions, cfg.radius_partitions))
    vecs = (Blur_Vector * (10 * n))()
    P = ctypes.POINTER(ctypes.c_double)

    def run():
        if lib.phd_blur_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), bins.ctypes.data_as(P), vecs,
                                     None) != 0:
            raise RuntimeError(f"blur batch failed: {last_error()}")
    run()
    lib.phd_profile_kernels(0)
    lib.phd_profile_kernels(0b110 | (4 << 24))      # rows and columns, every 4th call
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    wall = (time.perf_counter() - t0) / iters
    us = {}
    for k, name in ((1, "fft_rows"), (2, "fft_cols")):
        tot, cnt = ctypes.c_double(), ctypes.c_long()
        lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
        us[name] = 1000 * tot.value / max(cnt.value, 1)
    lib.phd_profile_kernels(0)
    del t
    torch.cuda.empty_cache()
    wf = w // 2 + 1
    ab = 18.0 * h * wf
    return {"workload": f"{n} x {h}x{w} RGB8, FFT + blur_profile only, device-resident",
            "images_per_s": round(n / wall, 1), "ms_per_batch_wall": round(1000 * wall, 3),
            "kernel_us_per_image": {k: round(v, 2) for k, v in us.items()},
            "roofline": {"kernel": "fft_cols", "bound": "hbm", "achieved": round(ab / (us["fft_cols"] * 1e-6) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ab / (us["fft_cols"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": ab, "avg_launch_us": round(us["fft_cols"], 2)}}


def config5(lib, last_error, n=512, iters=2):
    """BASELINE config 5 on one GPU: full reports of n device-resident images of
    mixed sizes (shard.MIXED_SHAPES, 512^2 .. 6000x4000; 512 is one rank's share
    of the 4096 at 8 GPUs) with h/s/v = 36/4/5, through
    phd_report_batch_device_mixed (one batched run per size group)."""
    import torch
    from photohive_dsp_amd import shard
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    sizes = shard.mixed_sizes(n, 5)
    ts = []
    for i, (h, w) in enumerate(sizes):
        t = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
        assert lib.phd_fill_uniform_device(t.data_ptr(), t.numel(), 5000 + i, None) == 0, last_error()
        ts.append(t)
    cfg = make_config(h_partitions=36, s_partitions=4, v_partitions=5)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    hs = (ctypes.c_int * n)(*[h for h, _ in sizes])
    ws = (ctypes.c_int * n)(*[w for _, w in sizes])
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()

    def run():
        if lib.phd_report_batch_device_mixed(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st, None) != 0:
            raise RuntimeError(f"mixed batch failed: {last_error()}")
        for i in range(n):
            r = outs[i]
            lib.free_full_report(ctypes.byref(r))
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    wall = (time.perf_counter() - t0) / iters
    mpx = sum(h * w for h, w in sizes) / 1e6
    del ts
    torch.cuda.empty_cache()
    return {"workload": f"{n} mixed-size RGB8 images (seed 5, {len(set(sizes))} sizes, {mpx:.0f} Mpx), "
                        "full report, h/s/v 36/4/5, device-resident",
            "images_per_s": round(n / wall, 1), "megapixels_per_s": round(mpx / wall, 1),
            "ms_per_batch_wall": round(1000 * wall, 2)}


def algorithmic_bytes(kernel, h, w):
    """Bytes one launch must move: RGB8 reads of the pixel passes,
    the fp64-complex half spectrum written by the row pass and read by the column
    pass, which also reads the u16 polar-bin map (2 B per spectrum element)."""
    n, hwf = h * w, h * (w // 2 + 1)
    return {"hsv_stats": 3 * n, "palette_sums": 3 * n, "fft_rows": 3 * n + 16 * hwf,
            "fft_cols": 18 * hwf}.get(kernel)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    # PHD_BENCH_BACKEND=gloo rehearses the N>1 path with several ranks on one
    # GPU (RCCL refuses two ranks on one device); the driver's runs use nccl
    backend = os.environ.get("PHD_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = local % ndev if ndev else local
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    import photohive_dsp_amd  # noqa: F401
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.lib import last_error, lib
    from photohive_dsp_amd.structures import Full_Report_Data

    H, W, B = args.height, args.width, args.batch
    img_bytes = H * W * 3
    d_imgs = torch.empty(B * img_bytes, dtype=torch.uint8, device="cuda")
    for i in range(B):
        seed = rank * B + i
        sub = d_imgs[i * img_bytes:(i + 1) * img_bytes]
        assert lib.phd_fill_uniform_device(sub.data_ptr(), img_bytes, seed, None) == 0, last_error()
    torch.cuda.synchronize()
    cfg = make_config()
    outs = (ctypes.POINTER(Full_Report_Data) * B)()
    status = (ctypes.c_int * B)()

    def step():
        rc = lib.phd_report_batch_device(d_imgs.data_ptr(), B, H, W, img_bytes, ctypes.byref(cfg), outs,
                                         status, None)
        if rc != 0:
            raise RuntimeError(f"report batch failed ({rc}): {last_error()}")
        for i in range(B):
            lib.free_full_report(ctypes.byref(outs[i]))

    from photohive_dsp_amd.lib import KERNELS

    def kernel_times():
        out = {}
        for k, name in enumerate(KERNELS):
            tot, cnt = ctypes.c_double(), ctypes.c_long()
            lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
            if cnt.value:
                out[name] = {"total_ms": tot.value, "launches": cnt.value, "avg_us": 1000 * tot.value / cnt.value}
        return out

    # warmup; the last warmup step with events on every kernel, to find the
    # dominant one in steady state
    lib.phd_profile_kernels(0)
    for _ in range(max(1, args.warmup) - 1):
        step()
    lib.phd_profile_kernels(0 if args.no_kernel_events else (1 << len(KERNELS)) - 1)
    step()
    warm = kernel_times()
    dom = max(warm, key=lambda k: warm[k]["total_ms"]) if warm else None

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    # timed region: HIP events bracket every launch of the dominant kernel in
    # every 4th step (bracketing every launch of every step costs ~6% throughput)
    lib.phd_profile_kernels(0 if dom is None else (1 << KERNELS.index(dom)) | (4 << 24))
    barrier()
    t0 = time.perf_counter()
    stage = [0.0] * 8
    for _ in range(args.steps):
        step()
        tm = (ctypes.c_double * 8)()
        lib.phd_last_timings(tm, 8)
        for j in range(8):
            stage[j] += tm[j]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern = kernel_times()

    # the single collective: max of wall time, sums of images / pixels (shard.py)
    from photohive_dsp_amd.shard import merge_counters
    elapsed, images, _ = merge_counters(elapsed, float(B * args.steps), float(B * args.steps * H * W),
                                        device="cuda" if backend == "nccl" else "cpu")
    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    value = images / elapsed
    line = {
        "metric": "images/sec (4000\u00d73000 RGB8 full report) at 1/2/4/8 GPUs; HBM GB/s vs peak",
        "value": round(value, 3),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (device splitmix64 uniform RGB8)",
        "config": {"workload": f"full report, {H}x{W} RGB8, batch {B}/GPU, device-resident",
                   "global_batch": B * world, "image": f"{H}x{W}", "parallelism": f"images sharded over {world} GPU"},
        "stages_ms_per_step": {"hsv_stats": stage[0] / args.steps, "fft_rows_cols": stage[1] / args.steps,
                               "palette_pass2": stage[2] / args.steps, "gpu_total": stage[3] / args.steps,
                               "host_total": stage[4] / args.steps, "host_enqueue": stage[5] / args.steps,
                               "host_decisions": stage[6] / args.steps, "host_assembly": stage[7] / args.steps},
    }
    line["roofline"] = None
    if dom in kern:
        # the palette passes take the whole batch in one launch, the FFT passes one image
        # (from the last warmup step, whose every launch was bracketed)
        per_launch = B / warm[dom]["launches"]
        ab = algorithmic_bytes(dom, H, W) * per_launch
        achieved = ab / (kern[dom]["avg_us"] * 1e-6) / 1e9
        traffic = None
        try:
            with open(args.pmc) as f:
                pm = json.load(f)
            if pm.get("image") == f"{H}x{W}" and dom in pm.get("kernels", {}):
                traffic = pm["kernels"][dom]["hbm_bytes_per_image"] * per_launch
        except (OSError, ValueError, KeyError):
            pass
        line["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1),
                            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                            "traffic": traffic, "algorithmic_bytes_per_launch": ab,
                            "images_per_launch": per_launch,
                            "avg_launch_us": round(kern[dom]["avg_us"], 2),
                            "launches_timed": kern[dom]["launches"], "sampling": "every launch of every 4th step"}
        line["warmup_kernels_us_per_launch"] = {k: round(v["avg_us"], 2) for k, v in warm.items()}
    if not args.no_config3 and world == 1:
        line["config2_single"] = single_image(lib, last_error, H, W)
        line["config3"] = config3(lib, last_error)
        line["config4"] = config4(lib, last_error)
        line["config5"] = config5(lib, last_error)
    if not args.no_cpu_baseline and world == 1:     # rank 0 at N=1 only
        line["cpu_baseline"] = cpu_baseline(H, W, args.cpu_images)
    print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
