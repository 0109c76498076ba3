"""Benchmark: images/s of the full PhotoHive_DSP report on 4000x3000 RGB8 images
(BASELINE.json config 2 at N=1; weak-scaled batches per GPU for N>1), plus the
other BASELINE configs as objects of the same JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

`--gpus N` without a torchrun environment starts the N ranks itself (a
torchrun child process, before this process touches the GPU) and exits with
its status.  One process per GPU; rank r uses device r (backend "nccl" = RCCL;
PHD_BENCH_BACKEND=gloo rehearses N ranks on one GPU).

A step = one full report (stats, S-bar, palette, blur profile, blur vectors)
of every image of one device-resident batch of B images per GPU.  Images are
synthetic (splitmix64 uniform RGB8, generated on the device; seed = global
image index).  Ranks shard images with no data-path collective; one small
all-reduce merges the counters (shard.merge_counters).  Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "images/sec (4000×3000 RGB8 full report) at 1/2/4/8 GPUs; HBM GB/s vs peak"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--batch", type=int, default=512,
                   help="images per GPU per step (one lane: 6.7k images/s at 16, 7.0k at 32-48, 7.1k at 64, "
                        "7.0-7.3k at 128, 7.4k at 256 on one box (round 3); two lanes, 8 queues: 8.70-8.72k at 256, "
                        "8.80k at 512 (round 4): the per-call fixed costs -- K1's prologue and tail, the host head "
                        "and tail of a call -- amortised; 18.4 GB of pixels)")
    p.add_argument("--lanes", type=int, default=2,
                   help="library lanes for every config of the run (phd_set_lanes; 2 is the library's default: "
                        "each call split into two concurrent halves, +10-13 %% images/s over 1).  With 2 the "
                        "headline roofline is the whole pipeline's and one_lane repeats the headline on one "
                        "lane, where each launch of the dominant kernel runs alone and its events price it")
    p.add_argument("--hw-queues", type=int, default=8,
                   help="GPU_MAX_HW_QUEUES for this process (set before HIP initialises; 0 keeps the environment's, "
                        "HIP's own default is 4): two lanes drive 4 HIP streams beside HIP's copy traffic (round 5: "
                        "8.60-8.77k images/s with HIP's 4 queues, 8.87-8.97k with 8)")
    p.add_argument("--no-one-lane", action="store_true",
                   help="skip the one-lane repeat of the headline (one_lane)")
    p.add_argument("--height", type=int, default=3000)
    p.add_argument("--width", type=int, default=4000)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-procs", type=int, default=0,
                   help="CPU baseline processes (0: the affinity set, bounded by the cgroup quota and the box's "
                        "per-GPU CPU share; cpu_topology)")
    p.add_argument("--no-kernel-events", action="store_true",
                   help="do not bracket kernels with HIP events (roofline then null)")
    p.add_argument("--no-configs", "--no-config3", dest="no_configs", action="store_true",
                   help="headline only: skip the BASELINE config 3/4/5 objects and the host-buffer runs")
    p.add_argument("--config4-images", type=int, default=2048, help="config 4 total images (all ranks)")
    p.add_argument("--config5-images", type=int, default=4096, help="config 5 total images (all ranks)")
    p.add_argument("--plan-only", action="store_true",
                   help="no GPU: start the ranks, shard configs 2/4/5 and merge the counters (gloo), print the plan")
    p.add_argument("--plan-visible-devices", type=int, default=None,
                   help="--plan-only: devices the ranks would see (default: torch.cuda.device_count(); 1 rehearses "
                        "several ranks on one card, which the line then reports as n_gpus 1)")
    p.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                   help="per-kernel PMC traffic summary written by tools/pmc_collect.py")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------
# N ranks from a plain `python bench.py --gpus N`
# ---------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args, argv=None) -> int:
    """Start `torch.distributed.run` with N ranks as a CHILD process (nothing in
    this process has touched the GPU) and return its exit status."""
    argv = sys.argv[1:] if argv is None else argv
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


# ---------------------------------------------------------------------------
# CPU baseline (rank 0 at N=1, before the GPU is touched)
# ---------------------------------------------------------------------------
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _fft_engine():
    import ctypes.util
    fftw = ctypes.util.find_library("fftw3")
    try:
        import scipy
        eng = f"scipy.fft.rfft2 (pocketfft, scipy {scipy.__version__})"
    except ImportError:
        eng = "numpy.fft.rfft2"
    return eng + ("" if fftw is None else f"; libfftw3 present ({fftw}) but not used")


def _cgroup_cpu_max():
    """The cgroup v2 CPU quota of this process ("max 100000" = none), or None."""
    for p in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            pass
    try:                                                   # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = f.read().strip()
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            return f"{'max' if q == '-1' else q} {f.read().strip()}"
    except OSError:
        return None


def _physical_cores(cpus):
    """Distinct physical cores among the logical CPUs `cpus` (SMT siblings once)."""
    seen = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                seen.add(f.read().strip())
        except OSError:
            seen.add(str(c))
    return len(seen)


def cpu_topology():
    """What this process may run on (P = the host's CPUs), and the
    process count the baseline uses: the affinity set, bounded by the cgroup quota
    and by the CPU share the GPU box grants one GPU's job (OMP_NUM_THREADS there:
    worker pools are to be sized to it), with the reason recorded."""
    aff = sorted(os.sched_getaffinity(0))
    quota = _cgroup_cpu_max()
    quota_cpus = None
    if quota and not quota.startswith("max"):
        q, per = quota.split()[:2]
        quota_cpus = max(1, -(-int(q) // int(per)))
    share = os.environ.get("OMP_NUM_THREADS")
    share = int(share) if share and share.isdigit() and int(share) > 0 else None
    procs, why = len(aff), "every CPU in sched_getaffinity"
    if quota_cpus is not None and quota_cpus < procs:
        procs, why = quota_cpus, f"cgroup cpu.max quota {quota} allows {quota_cpus} CPUs"
    if share is not None and share < procs:
        procs, why = share, (f"the GPU box grants one GPU's job a share of {share} CPUs (OMP_NUM_THREADS={share}; "
                             f"its rules size worker pools to that share), of {len(aff)} in the affinity set")
    return {"affinity_cpus": len(aff), "affinity_physical_cores": _physical_cores(aff),
            "host_cpus_online": os.sysconf("SC_NPROCESSORS_ONLN"), "cgroup_cpu_max": quota,
            "cpu_share_env": share, "procs": procs, "procs_reason": why}


def _cpu_worker(job):
    """One baseline process: the oracle build `opt` on its own images."""
    opt, h, w, seeds, start_at, fft_workers = job
    from oracle import oracle as orc
    from photohive_dsp_amd import synth
    orc.use_build(opt)
    orc.report(synth.uniform(400, 400, 1))                 # load the library outside the timing
    imgs = [synth.uniform(h, w, s) for s in seeds]
    while time.time() < start_at:
        time.sleep(0.005)
    t0 = time.time()
    for im in imgs:
        orc.report(im, fft_workers=fft_workers)
    return len(imgs), t0, time.time()


def _throughput(h, w, procs, per, seed0):
    """`procs` processes, `per` images each, common start: (images, wall s)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        start_at = time.time() + 5.0 + 0.2 * procs
        jobs = [("O2", h, w, [seed0 + per * p + k for k in range(per)], start_at, 1) for p in range(procs)]
        res = pool.map(_cpu_worker, jobs, chunksize=1)
        # the workers exit on their own (the with-block's terminate() would
        # SIGTERM them, which a profiler wrapping the run reports per process)
        pool.close()
        pool.join()
    return sum(r[0] for r in res), max(r[2] for r in res) - min(r[1] for r in res)


def cpu_baseline(h, w, topo, procs):
    """BASELINE.md 3 / SURVEY.md 8(d): the C restatement of the reference path
    (oracle/phd_oracle.c + scipy rfft2 for FFTW), u8 host buffer -> full report,
    on this host's cores.  Throughput mode (the `value`): `procs` independent
    processes (the reference is not reentrant), one image at a time each, -O2;
    the same at half the processes shows whether the rate scales with cores.
    Latency mode: one image at a time with the FFT on `procs` threads (the
    reference plans FFTW with sysconf(_SC_NPROCESSORS_ONLN) threads,
    src/utilities.c:128, src/fft_processing.c:21), at -O2 and at -O0 (the
    reference ships -O0)."""
    from oracle import oracle as orc
    from photohive_dsp_amd import synth
    orc.build()                                            # liboracle.so + liboracle_O0.so (no-op when built)
    out = {"unit": "images/s", "kind": "port", "cores": procs, **topo, "cpu_model": _cpu_model(),
           "fft_engine": _fft_engine()}
    # latency mode: one image at a time, FFT on all `procs` cores
    lat = {}
    for opt, n in (("O2", 3), ("O0", 2)):
        orc.use_build(opt)
        orc.report(synth.uniform(400, 400, 1))
        imgs = [synth.uniform(h, w, 20_000 + i) for i in range(n)]
        t0 = time.perf_counter()
        for im in imgs:
            orc.report(im, fft_workers=procs)
        dt = time.perf_counter() - t0
        lat[opt] = {"ms_per_image": round(1000 * dt / n, 1), "images_per_s": round(n / dt, 3),
                    "sample": f"{n} x {h}x{w} uniform, one at a time"}
    # BASELINE config 1: one 1024x1024 uniform image (splitmix64 seed 20241125,
    # tests/golden/uniform_1024.npz pins the report), one call at a time
    c1 = {}
    img1 = synth.uniform(1024, 1024, 20241125)
    for opt in ("O2", "O0"):
        orc.use_build(opt)
        orc.report(img1, fft_workers=procs)
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            orc.report(img1, fft_workers=procs)
            ts.append(time.perf_counter() - t0)
        c1[f"ms_{opt}"] = round(1000 * sorted(ts)[1], 2)
    out["config1"] = {"workload": "1 x 1024x1024 uniform RGB8 (seed 20241125), full report, median of 3", **c1}
    orc.use_build("O2")
    # throughput mode: `procs` processes, 2 images each, common start; then half
    # as many processes (does the rate scale with the cores used?)
    per = 2
    n_img, wall = _throughput(h, w, procs, per, 30_000)
    out["value"] = round(n_img / wall, 3)
    out["mode"] = "throughput"
    out["per_core_images_per_s"] = round(n_img / wall / procs, 4)
    out["sample"] = (f"{procs} processes x {per} x {h}x{w} uniform RGB8 full reports (-O2 restatement, "
                     f"1 FFT thread each): {n_img} images in {wall:.1f} s wall")
    half = max(1, procs // 2)
    n_h, wall_h = _throughput(h, w, half, per, 40_000)
    scal = (n_img / wall) / (n_h / wall_h) / (procs / half) if half < procs else 1.0
    out["modes"] = {"throughput_O2": {"images_per_s": out["value"], "processes": procs},
                    f"throughput_O2_{half}_procs": {"images_per_s": round(n_h / wall_h, 3), "processes": half},
                    "scaling_efficiency_half_to_full": round(scal, 3),
                    "latency_O2": lat["O2"], "latency_O0": lat["O0"]}
    # what the whole affinity set would give if the per-core rate held (a
    # projection, not a measurement: more processes than the granted share are
    # not run on the shared box)
    out["projected_affinity_images_per_s"] = round(out["per_core_images_per_s"] * topo["affinity_physical_cores"], 2)
    out["projection_basis"] = ("per_core_images_per_s x affinity_physical_cores (one process per physical core; "
                               "assumes the per-core rate measured at `cores` processes holds)")
    return out


# ---------------------------------------------------------------------------
# GPU configs
# ---------------------------------------------------------------------------
def algorithmic_bytes(kernel, h, w):
    """Bytes one launch must move per image: RGB8 reads of the pixel
    passes, the fp64-complex half spectrum written by the row pass and read by the
    column pass (its polar-bin runs, ~1.5 MB per size shared by every image, are
    an implementation table, not counted)."""
    n, hwf = h * w, h * (w // 2 + 1)
    # report_design: the bytes this build's report moves -- SURVEY 8(d)'s 9 N
    # counts a second RGB8 read for the palette's calculate_avg_hsv pass, which
    # the one-pass palette (K1 sums h / s / v per hue cell) does not make; the
    # tie-overflow walk (k_partial_sums_img) reads only a prefix of some images
    return {"hsv_stats": 3 * n, "palette_sums": 3 * n, "fft_rows": 3 * n + 16 * hwf,
            "fft_cols": 16 * hwf, "blur_path": 3 * n + 32 * hwf, "report": 9 * n + 32 * hwf,
            "report_design": 6 * n + 32 * hwf}[kernel]


def per_kernel_roofline(warm, B, H, W):
    """Each per-image pass's HBM fraction from the warm-up steps that bracket
    its launches (one kernel per step): algorithmic bytes per
    launch / average launch time / peak."""
    out = {}
    for name, v in warm.items():
        per_launch = B / v["launches"]
        ab = algorithmic_bytes(name, H, W) * per_launch
        gbs = ab / (v["avg_us"] * 1e-6) / 1e9
        out[name] = {"avg_launch_us": round(v["avg_us"], 2), "images_per_launch": per_launch,
                     "us_per_image": round(v["avg_us"] / per_launch, 2),
                     "algorithmic_bytes_per_image": algorithmic_bytes(name, H, W),
                     "achieved_GB_per_s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    return out


def pipeline_roofline(images_per_s, H, W):
    """The whole report against HBM: images/s x SURVEY.md 8(d)'s 9 N + 32 H Wf
    bytes (`frac`), and beside it on the bytes this design moves, 6 N + 32 H Wf
    (`frac_design_bytes`: no second RGB8 pass for the palette sums)."""
    gbs = images_per_s * algorithmic_bytes("report", H, W) / 1e9
    gbs_d = images_per_s * algorithmic_bytes("report_design", H, W) / 1e9
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_image": algorithmic_bytes("report", H, W),
            "achieved_design_bytes": round(gbs_d, 1), "frac_design_bytes": round(gbs_d / HBM_PEAK_GBS, 4),
            "design_bytes_per_image": algorithmic_bytes("report_design", H, W),
            "design_bytes_note": "SURVEY 8(d)'s 9N + 32HWf less the 3N palette pass-2 re-read this build does not "
                                 "make (K1 sums h/s/v per hue cell in its one pass)"}


def pmc_traffic(args, H, W):
    """The per-kernel HBM bytes of the committed PMC passes (tools/pmc_collect.py)
    for this image size, with where they come from; (None, None) without them."""
    try:
        with open(args.pmc) as f:
            pm = json.load(f)
    except (OSError, ValueError):
        return None, None
    if pm.get("image") != f"{H}x{W}" or not pm.get("kernels"):
        return None, None
    src = (f"{os.path.relpath(args.pmc, ROOT)}: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this "
           "config (tools/pmc_collect.py), not measured in this run")
    if pm.get("bench_args"):
        src += (f"; profiled run: bench.py {' '.join(pm['bench_args'])}"
                + (f", {pm['images_profiled']} images" if pm.get("images_profiled") else ""))
    if pm.get("calibration"):
        src += f"; FETCH_SIZE x each kernel's fetch_factor, calibrated on its algorithmic bytes ({pm['calibration']})"
    return pm["kernels"], src


def dominant_roofline(hl, args):
    """The dominant kernel against HBM: its algorithmic bytes per launch over its
    average launch duration, from the HIP events of the timed region (every
    launch of every 4th step, all ranks; one lane, so each launch runs alone)."""
    H, W, B = args.height, args.width, args.batch
    m, dom, warm, kern = hl["merged"], hl["dom"], hl["warm"], hl["kern"]
    if dom not in kern:
        return None
    # the palette passes take the whole batch in one launch, the FFT passes one image
    per_launch = hl["warm_steps"] * B / warm[dom]["launches"]
    ab = algorithmic_bytes(dom, H, W) * per_launch
    avg_us = 1000 * m["kernel_ms"] / max(m["launches"], 1)      # all ranks' sampled launches
    achieved = ab / (avg_us * 1e-6) / 1e9
    kt, tsrc = pmc_traffic(args, H, W)
    traffic = kt[dom]["hbm_bytes_per_image"] * per_launch if kt and dom in kt else None
    return {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": tsrc if traffic else None, "algorithmic_bytes_per_launch": ab,
            "images_per_launch": per_launch, "avg_launch_us": round(avg_us, 2), "launches_timed": int(m["launches"]),
            "sampling": "every launch of every 4th timed step, all ranks"}


def pipeline_headline_roofline(value, hl, args):
    """Two or more lanes: the launches of the lanes overlap, so no one kernel's
    duration prices it; the headline roofline is the whole report's --
    SURVEY.md 8(d)'s 9 N + 32 H Wf bytes per image x the timed region's images/s
    (its wall clock, all ranks) -- with the PMC bytes of every kernel of the
    report summed per image as traffic.  dominant_kernel_shared: the column
    pass's events in a warm-up step on those lanes (shared launches); one_lane.roofline
    has it alone."""
    H, W, B = args.height, args.width, args.batch
    out = pipeline_roofline(value, H, W)
    out = {"kernel": f"report pipeline (hsv_stats + fft_rows + fft_cols + palette passes, {hl['lanes']} lanes)",
           **out}
    kt, tsrc = pmc_traffic(args, H, W)
    if kt:
        out["traffic"] = round(sum(v["hbm_bytes_per_image"] for v in kt.values()))
        out["traffic_source"] = tsrc + f"; summed over {sorted(kt)} per image"
        out["traffic_per"] = "image"
    else:
        out["traffic"] = None
    out["basis"] = "images/s of the timed region x algorithmic bytes per image"
    dom, warm = hl["dom"], hl["warm"]
    if dom in warm:
        per_launch = B / warm[dom]["launches"]
        gbs = algorithmic_bytes(dom, H, W) * per_launch / (warm[dom]["avg_us"] * 1e-6) / 1e9
        out["dominant_kernel_shared"] = {"kernel": dom, "avg_launch_us": round(warm[dom]["avg_us"], 2),
                                         "achieved": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                                         "source": "HIP events on every launch of one warm-up step on the same lanes"}
    return out


class Ctx:
    """Per-rank state shared by the configs."""

    def __init__(self, args, world, rank, backend, dev=None):
        import torch
        from photohive_dsp_amd.lib import last_error, lib
        self.args, self.world, self.rank, self.backend = args, world, rank, backend
        self.dev = dev            # this rank's device index (n_gpus = distinct devices over the ranks)
        self.torch, self.lib, self.last_error = torch, lib, last_error

    def barrier(self):
        if self.world > 1:
            self.torch.distributed.barrier()
        self.torch.cuda.synchronize()

    def merge(self, elapsed, images, pixels, alg_bytes, kernel_ms=0.0, launches=0.0):
        from photohive_dsp_amd.shard import merge_counters
        return merge_counters([elapsed, images, pixels, alg_bytes, kernel_ms, launches],
                              device="cuda" if self.backend == "nccl" else "cpu", dev_index=self.dev)

    def fill(self, t, seed):
        assert self.lib.phd_fill_uniform_device(t.data_ptr(), t.numel(), seed, None) == 0, self.last_error()


def kernel_times(lib, names):
    out = {}
    for k, name in enumerate(names):
        tot, cnt = ctypes.c_double(), ctypes.c_long()
        lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
        if cnt.value:
            out[name] = {"total_ms": tot.value, "launches": cnt.value, "avg_us": 1000 * tot.value / cnt.value}
    return out


def headline(cx, timed_events=True, kind="uniform", steps=None):
    """Config 2, weak-scaled: B device-resident 4000x3000 images per rank per step.
    timed_events=False: no kernel events in the timed region (the warm-up
    steps still time the candidates).  kind "hblur": SURVEY.md 8(d) row 2(b)'s
    structured images (gradient + disks + 15-px horizontal box blur, synth.py,
    generated on the device; seed 2 + global image index) instead of uniform
    random bytes."""
    args, lib, torch = cx.args, cx.lib, cx.torch
    steps = args.steps if steps is None else steps
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.lib import KERNELS
    from photohive_dsp_amd.structures import Full_Report_Data
    H, W, B = args.height, args.width, args.batch
    img_bytes = H * W * 3
    d_imgs = torch.empty(B * img_bytes, dtype=torch.uint8, device="cuda")
    for i in range(B):
        if kind == "hblur":
            assert lib.phd_fill_structured_device(d_imgs[i * img_bytes:].data_ptr(), H, W, 2 + cx.rank * B + i, 15, 1,
                                                  None) == 0, cx.last_error()
        else:
            cx.fill(d_imgs[i * img_bytes:(i + 1) * img_bytes], cx.rank * B + i)
    torch.cuda.synchronize()
    cfg = make_config()
    outs = (ctypes.POINTER(Full_Report_Data) * B)()
    status = (ctypes.c_int * B)()

    def step():
        rc = lib.phd_report_batch_device(d_imgs.data_ptr(), B, H, W, img_bytes, ctypes.byref(cfg), outs,
                                         status, None)
        if rc != 0:
            raise RuntimeError(f"report batch failed ({rc}): {cx.last_error()}")
        lib.phd_free_reports(outs, B)

    # warmup, then one more step per kernel with events around that kernel's
    # launches only (as in the timed region: events around every launch of all
    # kernels shift time between them, and the row and column passes are
    # within ~15 %), to find the dominant kernel in steady state
    # The candidates are the three per-image passes (the palette tail runs once
    # per step, ~0.2 ms); the last warmup steps are the profiled ones.
    cand = [] if args.no_kernel_events else ["fft_cols", "fft_rows", "hsv_stats"][:max(1, args.warmup)]
    lanes = lib.phd_set_lanes(0)
    lib.phd_profile_kernels(0)
    for _ in range(max(1, args.warmup) - len(cand)):
        step()

    def time_candidates():
        out = {}
        for name in cand:
            lib.phd_profile_kernels(1 << KERNELS.index(name))
            step()
            out.update({n: v for n, v in kernel_times(lib, KERNELS).items() if n == name})
        lib.phd_profile_kernels(0)
        return out
    warm = time_candidates()
    # with two lanes each launch shares the GPU with the other lane's: the same
    # candidates once more on one lane price each kernel alone (per_kernel)
    warm_alone = warm
    if lanes > 1 and cand:
        lib.phd_set_lanes(1)
        # one untimed step first: a one-lane call may launch kernel forms the
        # two-lane steps did not (the column pass's prefetch form), whose
        # first launches load their code
        step()
        warm_alone = time_candidates()
        lib.phd_set_lanes(lanes)
        step()
    nprof = 1
    dom = max(warm, key=lambda k: warm[k]["total_ms"]) if warm else None
    # timed region, one lane: HIP events (recorded by the launches themselves,
    # on the stream the kernel runs on) bracket every launch of the dominant
    # kernel in every 4th step.  Two lanes: none (they cost ~3 % of the
    # throughput there; the headline roofline is then the pipeline's, priced on
    # the timed region's wall clock)
    if lanes > 1:
        timed_events = False
    lib.phd_profile_kernels(0 if dom is None or not timed_events else (1 << KERNELS.index(dom)) | (4 << 24))
    cx.barrier()
    t0 = time.perf_counter()
    stage = [0.0] * 8
    for _ in range(steps):
        step()
        tm = (ctypes.c_double * 8)()
        lib.phd_last_timings(tm, 8)
        for j in range(8):
            stage[j] += tm[j]
    cx.barrier()
    elapsed = time.perf_counter() - t0
    kern = kernel_times(lib, KERNELS)
    lib.phd_profile_kernels(0)
    n_img = B * steps
    km = kern[dom]["total_ms"] if dom in kern else 0.0
    kl = kern[dom]["launches"] if dom in kern else 0
    m = cx.merge(elapsed, n_img, n_img * H * W, n_img * algorithmic_bytes("report", H, W), km, kl)
    del d_imgs
    torch.cuda.empty_cache()
    res = {"merged": m, "dom": dom, "warm": warm, "warm_alone": warm_alone, "warm_steps": nprof, "kern": kern,
           "steps": steps, "lanes": lanes,
           "stages": {k: stage[j] / steps for j, k in enumerate(
               ("hsv_stats", "fft_rows_cols", "palette_pass2", "gpu_total", "host_total", "host_enqueue",
                "host_decisions", "host_assembly"))}}
    return res


def single_image(cx, h=3000, w=4000, iters=20):
    """BASELINE config 2 as literally stated: ONE 4000x3000 image per call.
    Median latency of a full report from a device-resident image
    (phd_report_batch_device, batch 1) and from a host buffer
    (phd_report_u8: one 36 MB H2D copy included)."""
    import numpy as np
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    nb = h * w * 3
    t = torch.empty(nb, dtype=torch.uint8, device="cuda")
    cx.fill(t, 77)
    host = t.cpu().numpy()
    cfg = make_config()
    out = (ctypes.POINTER(Full_Report_Data) * 1)()
    st = (ctypes.c_int * 1)()

    def dev():
        if lib.phd_report_batch_device(t.data_ptr(), 1, h, w, nb, ctypes.byref(cfg), out, st, None) != 0:
            raise RuntimeError(cx.last_error())
        lib.free_full_report(ctypes.byref(out[0]))

    def hst():
        r = lib.phd_report_u8(host.ctypes.data, h, w, 0, ctypes.byref(cfg), None)
        if not r:
            raise RuntimeError(cx.last_error())
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


def config1(cx, iters=20):
    """BASELINE config 1: one 1024x1024 uniform RGB8 image (splitmix64 seed
    20241125) through the Python caller's get_report (core.py:171; the
    reference's core.py:442-486), host buffer in -> Report out, median of
    `iters`.  Parity is the tests' (tests/golden/uniform_1024.npz)."""
    import numpy as np
    from photohive_dsp_amd import core, synth
    img = synth.uniform(1024, 1024, 20241125)
    core.get_report(img)
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        core.get_report(img)
        ts.append(time.perf_counter() - t0)
    return {"workload": "1 x 1024x1024 uniform RGB8 (seed 20241125), get_report() from a host buffer, "
                        f"median of {iters}", "gpu_get_report_ms": round(1000 * float(np.median(ts)), 3)}


def legacy_entry(cx, h=3000, w=4000, iters=5):
    """The reference's own binding path (lib.py:25-34, core.py:456-476): three
    planes of doubles k / 255.0 in host memory -> get_full_report_data ->
    Full_Report_Data (the planes' 288 MB H2D, the k/255 test and the RGB8
    pipeline on the device).  Median of `iters` calls; the Python-side
    pil_image_to_image_rgb (utils.py:30-46) is not included."""
    import numpy as np
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd.structures import Image_RGB
    nb = h * w * 3
    t = torch.empty(nb, dtype=torch.uint8, device="cuda")
    cx.fill(t, 4242)
    rgb = t.cpu().numpy().reshape(h, w, 3)
    del t
    planes = [np.ascontiguousarray(rgb[:, :, c]).ravel() / 255.0 for c in range(3)]
    P = ctypes.POINTER(ctypes.c_double)
    im = Image_RGB(height=h, width=w, r=planes[0].ctypes.data_as(P), g=planes[1].ctypes.data_as(P),
                   b=planes[2].ctypes.data_as(P))
    times = []
    for k in range(iters + 1):
        t0 = time.perf_counter()
        ptr = lib.get_full_report_data(ctypes.byref(im), None, 18, 2, 3, 0.1, 0.1, 0.95, 1000, 1, 40, 72,
                                       0.1, 0.9, 1.20, 0.3, 2)
        dt = time.perf_counter() - t0
        if not ptr:
            raise RuntimeError(cx.last_error())
        lib.free_full_report(ctypes.byref(ptr))
        if k:
            times.append(dt)
    times.sort()
    return {"workload": f"1 x {h}x{w} planar doubles k/255 (host) -> get_full_report_data, median of {iters}",
            "ms": round(1000 * times[len(times) // 2], 3)}


def host_buffers(cx, h=3000, w=4000, n=64, iters=3):
    """SURVEY.md 8(d)'s end-to-end timed region: u8 HOST buffers in ->
    Full_Report_Data out, through phd_report_batch_u8 (PCIe H2D included).
    Pageable numpy buffers, as a Python caller hands them over."""
    import numpy as np
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    nb = h * w * 3
    t = torch.empty(nb, dtype=torch.uint8, device="cuda")
    imgs = []
    for i in range(n):
        cx.fill(t, 9000 + i)
        imgs.append(t.cpu().numpy().copy())
    del t
    cfg = make_config()
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in imgs])
    hs = (ctypes.c_int * n)(*([h] * n))
    ws = (ctypes.c_int * n)(*([w] * n))
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()

    def run():
        if lib.phd_report_batch_u8(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st) != 0:
            raise RuntimeError(cx.last_error())
        lib.phd_free_reports(outs, n)
    run()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    wall = (time.perf_counter() - t0) / iters
    # the PCIe ceiling: pinned host -> device copies of the same bytes
    pin = torch.empty(16 * nb, dtype=torch.uint8).pin_memory()
    dst = torch.empty(16 * nb, dtype=torch.uint8, device="cuda")
    dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        dst.copy_(pin, non_blocking=True)
    torch.cuda.synchronize()
    pcie = 3 * 16 * nb / (time.perf_counter() - t0) / 1e9
    del pin, dst
    torch.cuda.empty_cache()
    eq = n * nb / wall / 1e9
    return {"workload": f"{n} x {h}x{w} RGB8 pageable host buffers -> reports (phd_report_batch_u8)",
            "images_per_s": round(n / wall, 1), "h2d_GB_per_s_equiv": round(eq, 2),
            "pinned_h2d_GB_per_s": round(pcie, 2), "frac_of_pinned_h2d": round(eq / pcie, 3),
            "ms_per_batch": round(1000 * wall, 2)}


def config3(cx, n=512, h=1080, w=1920, iters=10):
    """BASELINE config 3 (the HBM-roofline run): the rgb2hsv + rgb_statistics pass
    (phd_hsv_stats_batch_device, stats.hip) over n device-resident 1080p images, one
    launch per batch.  Kernel time from HIP events on the launch stream; algorithmic
    bytes = 3 per pixel."""
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd.structures import RGB_Statistics
    nb = h * w * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        cx.fill(t[i * nb:(i + 1) * nb], i)
    st = (RGB_Statistics * n)()
    sat = (ctypes.c_double * n)()

    def run():
        if lib.phd_hsv_stats_batch_device(t.data_ptr(), n, h, w, 0, st, sat, None) != 0:
            raise RuntimeError(f"hsv_stats batch failed: {cx.last_error()}")
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
    ab = float(n * algorithmic_bytes("hsv_stats", h, w))
    del t
    torch.cuda.empty_cache()
    return {"workload": f"{n} x {h}x{w} RGB8, rgb2hsv + rgb_statistics only, device-resident",
            "images_per_s": round(n / wall, 1), "ms_per_batch_wall": round(1000 * wall, 3),
            "roofline": {"kernel": "rgb_stats", "bound": "hbm", "achieved": round(ab / (us * 1e-6) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ab / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": ab, "avg_launch_us": round(us, 2)}}


def config4(cx, total, h=3000, w=4000, iters=3):
    """BASELINE config 4: `total` 4000x3000 images, FFT + blur-profile path alone
    (phd_blur_batch_device), sharded over the ranks with shard.assign (each rank
    one call over its device-resident share).  The column pass is this path's
    dominant kernel: its algorithmic bytes are the half spectrum it reads,
    16 * H * (W/2+1) per image (algorithmic_bytes("fft_cols");
    the whole path is 3N + 32 H Wf = 228 MB, the `alg_bytes` counter)."""
    import numpy as np
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd import shard
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Blur_Vector
    mine = shard.assign([(h, w)] * total, cx.world)[cx.rank]
    n = len(mine)
    nb = h * w * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for k, i in enumerate(mine):
        cx.fill(t[k * nb:(k + 1) * nb], 1000 + i)
    cfg = make_config()
    bins = np.zeros((n, cfg.angle_partitions, cfg.radius_partitions))
    vecs = (Blur_Vector * (10 * n))()
    P = ctypes.POINTER(ctypes.c_double)

    def run():
        if lib.phd_blur_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), bins.ctypes.data_as(P), vecs,
                                     None) != 0:
            raise RuntimeError(f"blur batch failed: {cx.last_error()}")
    run()
    lib.phd_profile_kernels(0)
    cx.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    cx.barrier()
    elapsed = (time.perf_counter() - t0) / iters
    # the kernel durations from one more pass with events on every row and
    # column launch (outside the timed passes: a pass is one call, so events
    # would otherwise bracket all of its launches), on one library lane so
    # each launch is timed alone on the GPU
    lanes = lib.phd_set_lanes(1)
    lib.phd_profile_kernels(0b110)
    run()
    lib.phd_set_lanes(lanes)
    us = {}
    for k, name in ((1, "fft_rows"), (2, "fft_cols")):
        tot, cnt = ctypes.c_double(), ctypes.c_long()
        lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
        us[name] = 1000 * tot.value / max(cnt.value, 1)
    lib.phd_profile_kernels(0)
    del t
    torch.cuda.empty_cache()
    m = cx.merge(elapsed, n, n * h * w, n * algorithmic_bytes("blur_path", h, w), us["fft_cols"] * n / 1000.0, n)
    ab = float(algorithmic_bytes("fft_cols", h, w))
    return {"workload": f"{total} x {h}x{w} RGB8 over {cx.world} GPU, FFT + blur_profile only, device-resident, "
                        f"{lanes} library lane(s)",
            "scaling": "strong", "n_gpus": m["devices"], "ranks": cx.world,
            "images_per_gpu_max": int(np.ceil(total / cx.world)),
            "images_per_s": round(m["images"] / m["elapsed"], 1),
            "ms_per_pass_wall": round(1000 * m["elapsed"], 3),
            "hbm_GB_per_s_path": round(m["alg_bytes"] / m["elapsed"] / 1e9, 1),
            "kernel_us_per_image_rank0": {k: round(v, 2) for k, v in us.items()},
            "roofline": {"kernel": "fft_cols", "bound": "hbm", "achieved": round(ab / (us["fft_cols"] * 1e-6) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(ab / (us["fft_cols"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": ab, "avg_launch_us": round(us["fft_cols"], 2)}}


def config5(cx, total, iters=4):
    """BASELINE config 5: `total` device-resident images of mixed sizes
    (shard.MIXED_SHAPES, 512^2 .. 6000x4000), full reports at h/s/v = 36/4/5,
    LPT-sharded by pixel count over the ranks (shard.assign), each rank one
    phd_report_batch_device_mixed call (one batched run per size group)."""
    lib, torch = cx.lib, cx.torch
    from photohive_dsp_amd import shard
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    sizes_all = shard.mixed_sizes(total, 5)
    mine = shard.assign(sizes_all, cx.world)[cx.rank]
    sizes = [sizes_all[i] for i in mine]
    n = len(mine)
    ts = []
    for i, (h, w) in zip(mine, sizes):
        t = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
        cx.fill(t, 5000 + i)
        ts.append(t)
    cfg = make_config(h_partitions=36, s_partitions=4, v_partitions=5)
    ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    hs = (ctypes.c_int * n)(*[h for h, _ in sizes])
    ws = (ctypes.c_int * n)(*[w for _, w in sizes])
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()

    def run():
        if lib.phd_report_batch_device_mixed(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st, None) != 0:
            raise RuntimeError(f"mixed batch failed: {cx.last_error()}")
        lib.phd_free_reports(outs, n)
    run()
    cx.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    cx.barrier()
    elapsed = (time.perf_counter() - t0) / iters
    pix = sum(h * w for h, w in sizes)
    ab = sum(algorithmic_bytes("report", h, w) for h, w in sizes)
    m = cx.merge(elapsed, n, pix, ab)
    del ts
    torch.cuda.empty_cache()
    return {"workload": f"{total} mixed-size RGB8 images (seed 5, {len(set(sizes_all))} sizes, "
                        f"{sum(h * w for h, w in sizes_all) / 1e6:.0f} Mpx) over {cx.world} GPU (LPT by pixels), "
                        f"full report, h/s/v 36/4/5, device-resident, {cx.lib.phd_set_lanes(0)} library lane(s)",
            "scaling": "strong", "n_gpus": m["devices"], "ranks": cx.world,
            "images_per_s": round(m["images"] / m["elapsed"], 1),
            "megapixels_per_s": round(m["pixels"] / m["elapsed"] / 1e6, 1),
            "hbm_GB_per_s_algorithmic": round(m["alg_bytes"] / m["elapsed"] / 1e9, 1),
            "ms_per_pass_wall": round(1000 * m["elapsed"], 2), "rank_elapsed_ms": [round(1000 * e, 2) for e in m["per_rank_elapsed"]]}


def plan_only(args, world, rank):
    """The multi-rank plumbing without a GPU (CPU tests): every rank takes its
    shard of configs 2, 4 and 5 exactly as the GPU run does and the counters
    are merged with the same single collective (gloo)."""
    import torch.distributed as dist
    from photohive_dsp_amd import shard
    if world > 1:
        dist.init_process_group("gloo")
    H, W, B = args.height, args.width, args.batch
    c4 = shard.assign([(H, W)] * args.config4_images, world)[rank]
    sizes5 = shard.mixed_sizes(args.config5_images, 5)
    c5 = shard.assign(sizes5, world)[rank]
    visible = args.plan_visible_devices
    if visible is None:
        import torch
        visible = torch.cuda.device_count()        # counts without initialising HIP
    dev = shard.device_of(int(os.environ.get("LOCAL_RANK", rank)), visible)
    out = {}
    for name, n, pix, ab in (("config2", B, B * H * W, B * algorithmic_bytes("report", H, W)),
                             ("config4", len(c4), len(c4) * H * W, len(c4) * algorithmic_bytes("blur_path", H, W)),
                             ("config5", len(c5), sum(sizes5[i][0] * sizes5[i][1] for i in c5),
                              sum(algorithmic_bytes("report", *sizes5[i]) for i in c5))):
        m = shard.merge_counters([1.0 + rank, n, pix, ab], dev_index=dev)
        out[name] = {"images": int(m["images"]), "pixels": int(m["pixels"]), "alg_bytes": int(m["alg_bytes"]),
                     "elapsed_max": m["elapsed"]}
    if rank == 0:
        print(json.dumps({"plan_only": True, "n_gpus": m["devices"], "ranks": world, **out}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def dump_maps(tag):
    """PHD_BENCH_MAPS=prefix: copy /proc/self/maps to prefix.<tag>.<pid> (crash
    triage: a native backtrace's raw addresses resolve against these mappings
    to library + offset, then addr2line / objdump on the same image)."""
    pre = os.environ.get("PHD_BENCH_MAPS")
    if pre:
        with open("/proc/self/maps") as f, open(f"{pre}.{tag}.{os.getpid()}", "w") as g:
            g.write(f.read())


def main(argv=None):
    args = parse(argv)
    if args.hw_queues > 0:
        # read by HIP when it initialises: before this process (or the ranks
        # spawn_ranks starts) makes any GPU call
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plan_only:
        return plan_only(args, world, rank)
    backend = os.environ.get("PHD_BENCH_BACKEND", "nccl")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before this process touches the GPU: the baseline's worker processes
        # start from a clean parent
        topo = cpu_topology()
        procs = args.cpu_procs or topo["procs"]
        if args.cpu_procs:
            topo["procs_reason"] = f"--cpu-procs {args.cpu_procs}"
        cpu = cpu_baseline(args.height, args.width, topo, procs)
    # the package before torch (its lib.py binds torch's HIP runtime file first)
    import photohive_dsp_amd  # noqa: F401
    import torch
    from photohive_dsp_amd import shard
    ndev = torch.cuda.device_count()
    dev = shard.device_of(local, ndev)
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    cx = Ctx(args, world, rank, backend, dev)
    if os.environ.get("PHD_BENCH_MAPS") and hasattr(cx.lib, "phd_install_crash_maps"):
        # the mappings AT a fault (SIGSEGV / SIGABRT ...), written by the library's handler
        cx.lib.phd_install_crash_maps(f"{os.environ['PHD_BENCH_MAPS']}.fault".encode())
    dump_maps("ctx")

    cx.lib.phd_set_lanes(args.lanes)                  # every config of this run
    hl = headline(cx)
    dump_maps("headline")
    extra = {}
    if hl["lanes"] > 1 and not args.no_one_lane:
        # the same workload on one lane: each launch alone on the GPU, so the
        # events in its timed region price the dominant kernel (the roofline of
        # the driver's contract); the headline's two lanes share the GPU
        cx.lib.phd_set_lanes(1)
        h1 = headline(cx)
        cx.lib.phd_set_lanes(args.lanes)
        if rank == 0:
            m1 = h1["merged"]
            extra["one_lane"] = {
                "workload": f"as the headline, each {args.batch}-image call on one library lane (phd_set_lanes(1))",
                "images_per_s": round(m1["images"] / m1["elapsed"], 1),
                "ms_per_step": round(1000 * m1["elapsed"] / h1["steps"], 3),
                "roofline": dominant_roofline(h1, args)}
    if not args.no_configs:
        # the same workload on structured images
        hs = headline(cx, timed_events=False, kind="hblur", steps=max(5, args.steps // 5))
        ms = hs["merged"]
        ips = ms["images"] / ms["elapsed"]
        extra["config2_structured"] = {
            "workload": f"full report, {args.height}x{args.width} RGB8 structured (synth.py hblur: gradient + disks "
                        f"+ 15-px horizontal box blur, generated on the device, seed 2 + image index), batch "
                        f"{args.batch}/GPU, {hs['lanes']} library lane(s), device-resident",
            "images_per_s": round(ips, 1), "ms_per_step": round(1000 * ms["elapsed"] / hs["steps"], 3),
            "steps": hs["steps"], "stages_ms_per_step_rank0": hs["stages"],
            "per_kernel": per_kernel_roofline(hs["warm_alone"], args.batch, args.height, args.width),
            "roofline_pipeline": pipeline_roofline(ips, args.height, args.width)}
        extra["config4"] = config4(cx, args.config4_images)
        extra["config5"] = config5(cx, args.config5_images)
        if world == 1:
            extra["config1"] = config1(cx)
            if cpu is not None and "config1" in cpu:
                extra["config1"]["cpu_ms_O2"] = cpu["config1"]["ms_O2"]
                extra["config1"]["cpu_ms_O0"] = cpu["config1"]["ms_O0"]
            extra["config2_single"] = single_image(cx, args.height, args.width)
            extra["host_buffer"] = host_buffers(cx, args.height, args.width)
            extra["legacy_entry"] = legacy_entry(cx, args.height, args.width)
            extra["config3"] = config3(cx)
    if rank == 0:
        m = hl["merged"]
        H, W, B = args.height, args.width, args.batch
        value = m["images"] / m["elapsed"]
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "images/s",
            "n_gpus": m["devices"],
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * m["elapsed"] / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device splitmix64 uniform RGB8)",
            "config": {"workload": f"full report, {H}x{W} RGB8, batch {B}/GPU, {hl['lanes']} library lane(s), "
                                   "device-resident",
                       "global_batch": B * world, "image": f"{H}x{W}",
                       "parallelism": f"images sharded over {world} rank(s) on {m['devices']} GPU"},
            "hbm_GB_per_s_algorithmic": round(m["alg_bytes"] / m["elapsed"] / 1e9, 1),
            "stages_ms_per_step_rank0": hl["stages"],
        }
        if hl["lanes"] > 1:
            line["roofline"] = pipeline_headline_roofline(value, hl, args)
        else:
            line["roofline"] = dominant_roofline(hl, args)
        line["warmup_kernels_us_per_launch"] = {k: round(v["avg_us"], 2) for k, v in hl["warm"].items()}
        line["per_kernel"] = per_kernel_roofline(hl["warm_alone"], B, H, W)
        line["roofline_pipeline"] = pipeline_roofline(value, H, W)
        line.update(extra)
        line["vs_baseline_note"] = ("null: BASELINE.md publishes no number for this metric (its only figures are "
                                    "per-stage CPU seconds on an unstated image size, README.md:62-75)")
        if cpu is not None:
            line["cpu_baseline"] = cpu
            # GPU / CPU ratios against the measured baseline and against the
            # whole-affinity projection (both images/s, 4000x3000 full reports)
            ratios = {"headline_device_resident": value}
            if "host_buffer" in extra:
                ratios["host_buffer"] = extra["host_buffer"]["images_per_s"]
            if "legacy_entry" in extra:
                ratios["legacy_entry"] = 1000.0 / extra["legacy_entry"]["ms"]
            line["vs_cpu_baseline"] = {
                k: {"images_per_s": round(v, 1), "x_measured": round(v / cpu["value"], 1),
                    "x_projected_affinity": round(v / cpu["projected_affinity_images_per_s"], 1)}
                for k, v in ratios.items()}
        print(json.dumps(line), flush=True)
    # the library's explicit teardown (threads joined, HIP resources released)
    # before torch's and HIP's own exit handlers; it would also run at exit
    if hasattr(cx.lib, "phd_shutdown"):                  # (older builds in A/B runs lack it)
        cx.lib.phd_shutdown()
    if world > 1:
        torch.distributed.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
