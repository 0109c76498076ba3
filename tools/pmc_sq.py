"""SQ/LDS counter passes for one pipeline kernel (run ON the GPU box).

    python tools/pmc_sq.py KERNEL [--iters N]     (KERNEL: 0 hsv_stats, 1 fft_rows, 2 fft_cols)
    python tools/pmc_sq.py 0 --probe 3000x4000:64   (tools/mixed_probe.py's full reports instead)

Each pass is a separate `rocprofv3 --pmc ...` run (counters only, no trace
domains) over tools/kbench.py; the per-kernel averages are printed and saved
to gpurun_out/pmc_sq_<kernel>.json.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_INSTS_VALU", "SQ_INSTS_LDS"],
    ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
     "SQ_INSTS_VMEM_WR", "GRBM_GUI_ACTIVE"],
    ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"],
]
NAMES = ["k_partial_sums", "k_k1t", "k_rgb_stats", "k_hsv_stats", "k_fft_rows", "k_fft_cols", "k_rows_ct", "k_cols_ct", "k_cutoffs", "k_palette_sums", "k_sharp"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("kernel", type=int)
    p.add_argument("--mask", default="0")
    p.add_argument("--probe", default="", help="SHAPE:N -- profile tools/mixed_probe.py N at PROBE_SHAPES=SHAPE")
    a = p.parse_args()
    target = [sys.executable, os.path.join(ROOT, "tools", "kbench.py"), str(a.kernel), a.mask]
    env = dict(os.environ)
    if a.probe:
        shape, n = a.probe.split(":")
        target = [sys.executable, os.path.join(ROOT, "tools", "mixed_probe.py"), n]
        env["PROBE_SHAPES"] = shape
    res = {}
    for i, counters in enumerate(PASSES):
        out = os.path.join(ROOT, "gpurun_out", f"pmcsq_{a.kernel}_{i}")
        cmd = ["rocprofv3", "--pmc"] + counters + ["--output-format", "csv", "-d", out, "-o", "p", "--"] + target
        try:
            r = subprocess.run(cmd, cwd=ROOT, env=env, timeout=150)
        except subprocess.TimeoutExpired:
            print(f"pass {i} timed out")
            break
        if r.returncode != 0:
            print(f"pass {i} failed rc={r.returncode}")
            continue
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        per = {}
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                short = next((n for n in NAMES if n in name), None)
                if short is None:
                    continue
                per.setdefault(short, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        for k, d in per.items():
            for c, v in d.items():
                res.setdefault(k, {})[c] = sum(v) / len(v)
    for k, d in res.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {v:16.1f}")
    with open(os.path.join(ROOT, "gpurun_out", f"pmc_sq_{a.kernel}.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
