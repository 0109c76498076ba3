"""Per-kernel HBM traffic from rocprofv3 PMC counters (run ON the GPU box).

Two separate counter passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on
gfx950's TCC slots), each with only --pmc (no trace domains), over the same
bench command.  Per MI355X_MICROARCH.md (HBM): bytes = counter * 1024, and
FETCH_SIZE reads half the bytes of wide coalesced streaming reads on gfx950,
so the read side is doubled.  Writes profiles/pmc_latest.json (+ a copy named
by --tag) for bench.py's roofline.traffic.

    python tools/pmc_collect.py --tag r06 -- --steps 1 --warmup 1 --batch 512 --lanes 2 --no-configs --no-one-lane
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = {"k_k1t": "hsv_stats", "k_rgb_stats": "rgb_stats", "k_hsv_stats": "hsv_stats", "k_fft_rows": "fft_rows", "k_fft_cols": "fft_cols",
         "k_rows_ct": "fft_rows", "k_cols_ct": "fft_cols", "k_cutoffs_b": "palette_cutoffs",
         "k_palette_sums_b": "palette_sums", "k_partial_sums_img": "palette_partial_sums",
         "k_partial_sums_b": "palette_partial_sums",
         "k_cutoffs": "palette_cutoffs", "k_palette_sums": "palette_sums", "k_sharp_pass": "sharpness"}


def short(name):
    for k, v in SHORT.items():
        if k + "(" in name or k + "<" in name or name.endswith(k):
            return v
    return None


def run_pass(counter, outdir, bench_args):
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-kernel-events"] + bench_args
    subprocess.run(cmd, check=True, cwd=ROOT)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {outdir}")
    per = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            k = short(row.get("Kernel_Name", ""))
            if not k or row.get("Counter_Name") != counter:
                continue
            per.setdefault(k, []).append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in per.items()}, files[0]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", default="latest")
    p.add_argument("--height", type=int, default=3000)
    p.add_argument("--width", type=int, default=4000)
    p.add_argument("rest", nargs=argparse.REMAINDER)
    a = p.parse_args()
    bench_args = [x for x in a.rest if x != "--"] + ["--height", str(a.height), "--width", str(a.width)]
    out = os.path.join(ROOT, "gpurun_out", "pmc")
    fetch, f1 = run_pass("FETCH_SIZE", out + "_fetch", bench_args)
    write, f2 = run_pass("WRITE_SIZE", out + "_write", bench_args)
    sys.path.insert(0, ROOT)
    from bench import parse as bench_parse
    ba = bench_parse(bench_args)
    # images profiled: one row-pass launch per image at the compile-time sizes
    # (every step of the run, warm-up and timing steps alike); the arithmetic
    # count as a fallback
    images = fetch["fft_rows"][1] if "fft_rows" in fetch else ba.batch * (ba.steps + max(1, ba.warmup))
    res = {"image": f"{a.height}x{a.width}", "source": [os.path.relpath(f1, ROOT), os.path.relpath(f2, ROOT)],
           "bench_args": bench_args, "images_profiled": images,
           "note": "rocprofv3 --pmc serialises kernel dispatches, so the two lanes' kernels (bench --lanes) ran one "
                   "at a time in these passes; each kernel's bytes per image are its own",
           "correction": "hbm_bytes = fetch_factor*FETCH_SIZE*1024 + WRITE_SIZE*1024 (fetch_factor 2 for streaming "
                         "reads, MI355X_MICROARCH.md; calibrated per FFT pass where profiles/pmc_calib.json has it)",
           "kernels": {}}
    # FETCH_SIZE -> bytes: x2 for 16-B-per-lane streaming reads (the guide's
    # calibration); the FFT passes' own patterns are calibrated on their
    # algorithmic bytes by tools/pmc_calib.py (profiles/pmc_calib.json)
    factors = {}
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_calib.json")) as f:
            cal = json.load(f)
        for kname, short_name in (("k_cols_ct", "fft_cols"), ("k_rows_ct", "fft_rows"), ("k_rgb_stats", "hsv_stats")):
            if kname in cal and cal.get("image") == f"{a.height}x{a.width}":
                factors[short_name] = cal[kname]["factor"]
        if factors:
            res["calibration"] = "profiles/pmc_calib.json (tools/pmc_calib.py)"
    except (OSError, ValueError, KeyError):
        pass
    for k in sorted(set(fetch) | set(write)):
        (fk, n), (wk, _) = fetch.get(k, (0.0, 0)), write.get(k, (0.0, 0))
        per_launch = images / max(n, 1)              # images per launch (< 1: several launches per image)
        fac = factors.get(k, 2.0)
        hbm = fac * fk * 1024 + wk * 1024
        res["kernels"][k] = {"fetch_size_kb": fk, "write_size_kb": wk, "launches": n, "fetch_factor": fac,
                             "images_per_launch": per_launch, "hbm_bytes_per_launch": hbm,
                             "hbm_bytes_per_image": hbm / per_launch,
                             "hbm_bytes_per_launch_x2": 2 * fk * 1024 + wk * 1024}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    # profiles/ for bench.py on this box; gpurun_out/ is what travels back
    for d, name in ((os.path.join(ROOT, "profiles"), "pmc_latest.json"),
                    (os.path.join(ROOT, "gpurun_out"), f"pmc_{a.tag}.json")):
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
