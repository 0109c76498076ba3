"""Print the key figures of a profiling round (run after tools/prof_round.sh)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def last_json(path):
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


def main():
    d = last_json(os.path.join(OUT, "bench_full.log"))
    r = d["roofline"]
    print("headline", d["value"], r["kernel"], r["frac"], r.get("dominant_kernel_shared"))
    if "one_lane" in d:
        o = d["one_lane"]
        print("one_lane", o["images_per_s"], o["roofline"]["kernel"], o["roofline"]["avg_launch_us"],
              o["roofline"]["frac"])
    print("config4", d["config4"]["images_per_s"], "config5", d["config5"]["images_per_s"])
    print("host_buffer", d["host_buffer"])
    print("config3 frac", d["config3"]["roofline"]["frac"], "single", d["config2_single"])
    for f in ("prof2", "prof"):
        path = os.path.join(OUT, f, "prof_kernel_stats.csv")
        if not os.path.exists(path):
            print(f, "no kernel statistics (", path, "missing )")
            continue
        for row in csv.DictReader(open(path)):
            if any(k in row["Name"] for k in ("k_cols_ct<3000", "k_rows_ct<4000", "k_k1t<512")):
                print(f, row["Name"][30:52], row["Calls"], round(float(row["AverageNs"]) / 1e3, 2))


if __name__ == "__main__":
    sys.exit(main())
