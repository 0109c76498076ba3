"""FETCH_SIZE / WRITE_SIZE of one FFT pass under ablation masks (run ON the
GPU box, ablate build): which part of the pass causes which memory traffic.
    python tools/pmc_masks.py KERNEL MASK [MASK ...]   (KERNEL 1 rows, 2 cols)
    (PMC_COUNTERS="TCC_EA0_RDREQ_sum ..." for other counters, one pass each)
-> gpurun_out/pmc_masks_K.json; per mask the average counter per launch of
tools/kbench.py's 20 timed launches (the first launch of each mask, the
setup report's, is dropped)."""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ABL = os.path.join(ROOT, "photohive_dsp_amd", "PhotoHive_DSP_lib", "libreport_data_ablate.so")
NAME = {1: "k_rows_ct", 2: "k_cols_ct"}


def run(counter, kernel, masks):
    out = os.path.join(ROOT, "gpurun_out", f"pmc_masks_{kernel}_{counter}")
    env = dict(os.environ, PHD_LIB=os.environ.get("PMC_LIB", ABL))
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "p", "--",
           sys.executable, os.path.join(ROOT, "tools", "kbench.py"), str(kernel)] + [str(m) for m in masks]
    subprocess.run(cmd, cwd=ROOT, env=env, check=True, timeout=170)
    f = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = []
    with open(f) as fh:
        rows = sorted(csv.DictReader(fh), key=lambda r: int(r.get("Dispatch_Id", 0)))
        for row in rows:
            if NAME[kernel] + "<" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    kernel = int(sys.argv[1])
    masks = [int(m) for m in sys.argv[2:]]
    res = {"kernel": NAME[kernel], "masks": {}}
    # PMC_COUNTERS="A B ...": other counters, one pass each (default the two sizes)
    for counter in os.environ.get("PMC_COUNTERS", "FETCH_SIZE WRITE_SIZE").split():
        v = run(counter, kernel, masks)
        per = len(v) // len(masks) if masks else 0     # launches per mask (setup report + 20 timed)
        for i, m in enumerate(masks):
            part = v[i * per:(i + 1) * per][1:]
            key = counter + ("_kb_avg" if counter.endswith("_SIZE") else "_avg")
            res["masks"].setdefault(str(m), {})[key] = sum(part) / max(len(part), 1)
            res["masks"][str(m)]["launches"] = len(part)
    with open(os.path.join(ROOT, "gpurun_out", f"pmc_masks_{kernel}.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
