"""FETCH_SIZE calibration of the FFT passes' own access patterns (run ON the
GPU box; MI355X_MICROARCH.md: only 16-B-per-lane streaming reads are
calibrated, other patterns must be calibrated on a known byte count).

Each pass is timed through phd_debug_time_kernel (tools/kbench.py) from the
ablation build (make -C photohive_dsp_amd/csrc ablate) with its compute
switched off, so the kernel moves exactly its algorithmic bytes; the ratio of
those bytes to FETCH_SIZE * 1024 is this pattern's counter factor.  The
production kernel's FETCH_SIZE times that factor is its read traffic.

    python tools/pmc_calib.py     -> gpurun_out/pmc_calib.json
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABL = os.path.join(ROOT, "photohive_dsp_amd", "PhotoHive_DSP_lib", "libreport_data_ablate.so")
H, W = 3000, 4000
WF = W // 2 + 1
KNOWN = {  # algorithmic read bytes per launch
    "k_cols_ct": 16 * H * (WF + 1),                     # tiles (phantom column included); the bin runs are ~1.5 MB
    "k_rows_ct": 3 * H * W,                             # RGB8
    "k_rgb_stats": 8 * 3 * H * W,                       # RGB8 of tools/stats_bench.py's 8-image launches
}
RUNS = [("k_cols_ct", 2, 0, False), ("k_cols_ct", 2, 1 | 2 | 16, True),
        ("k_rows_ct", 1, 0, False), ("k_rows_ct", 1, 1 | 2, True),
        # K1's per-lane dwordx3 pattern: the statistics pass reads each byte once
        ("k_rgb_stats", -1, 0, False)]


def fetch(kernel_id, mask, ablate_lib, tag):
    out = os.path.join(ROOT, "gpurun_out", f"pmc_calib_{tag}")
    env = dict(os.environ)
    if ablate_lib:
        env["PHD_LIB"] = ABL
    prog = ([os.path.join(ROOT, "tools", "stats_bench.py")] if kernel_id < 0 else
            [os.path.join(ROOT, "tools", "kbench.py"), str(kernel_id), str(mask)])
    cmd = ["rocprofv3", "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", out, "-o", "p", "--",
           sys.executable] + prog
    subprocess.run(cmd, cwd=ROOT, env=env, check=True, timeout=150)
    f = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            for k in KNOWN:
                if k + "<" in name and row.get("Counter_Name") == "FETCH_SIZE":
                    vals.setdefault(k, []).append(float(row["Counter_Value"]))
    return vals


def main():
    res = {"image": f"{H}x{W}", "known_read_bytes": KNOWN, "runs": {}}
    for i, (k, kid, mask, abl) in enumerate(RUNS):
        v = fetch(kid, mask, abl, f"{k}_{mask}")
        kb = v.get(k, [])
        # the timed launches (the report run before them has one launch per pass)
        avg = sum(kb[1:]) / max(len(kb) - 1, 1) if len(kb) > 1 else (kb[0] if kb else 0.0)
        res["runs"][f"{k} ablate {mask}"] = {"fetch_size_kb": avg, "launches": len(kb),
                                             "fetch_bytes_x1024": avg * 1024}
    for k in KNOWN:
        if k == "k_rgb_stats":
            moved = res["runs"].get(f"{k} ablate 0", {}).get("fetch_bytes_x1024")
            if moved:
                # applied to K1 (k_k1t), whose loads are the same 12-byte-per-lane pattern
                res[k] = {"factor": KNOWN[k] / moved, "applies_to": "k_k1t"}
            continue
        moved = res["runs"].get(f"{k} ablate {1 | 2 | 16 if k == 'k_cols_ct' else 1 | 2}", {}).get("fetch_bytes_x1024")
        prod = res["runs"].get(f"{k} ablate 0", {}).get("fetch_bytes_x1024")
        if moved and prod:
            f = KNOWN[k] / moved
            res[k] = {"factor": f, "production_read_bytes": prod * f, "vs_algorithmic": prod * f / KNOWN[k]}
    with open(os.path.join(ROOT, "gpurun_out", "pmc_calib.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
