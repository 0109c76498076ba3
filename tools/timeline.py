"""How the kernels of a bench run share the GPU in time, from a rocprofv3
kernel trace (run anywhere):

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o tl -- python bench.py --no-configs ...
    python tools/timeline.py gpurun_out/tl [--out profiles/r05/timeline.json]

Window: from the 3rd K1 (k_k1t) dispatch to the last one (whole steps of the
timed region; each lane launches one K1 per call).  Prints the window's
span, the time with 0 / 1 / 2 / 3+ kernels in flight, and per kernel name
its summed duration, its time alone on the GPU and its time beside another
kernel."""
import argparse
import collections
import csv
import glob
import gzip
import json
import os


def short(name):
    for k in ("k_k1t", "k_rows_ct", "k_cols_ct", "k_partial_sums_img", "k_cutoffs", "k_fft_rows", "k_fft_cols"):
        if k in name:
            return k
    n = name.replace("(anonymous namespace)", "anon").split("(")[0]
    return n.split("::")[-1][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f = (glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True) +
         glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv.gz"), recursive=True))[0]
    fh = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                  for r in csv.DictReader(fh))
    k1 = [r[0] for r in rows if r[2] == "k_k1t"]
    if len(k1) < 4:
        names = collections.Counter(r[2] for r in rows)
        raise SystemExit(f"{f}: {len(rows)} dispatches, K1 {len(k1)}; names {names.most_common(6)}")
    t0, t1 = k1[2], k1[-1]
    rows = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
    ev = []
    for i, (s, e, n) in enumerate(rows):
        ev.append((s, 1, i))
        ev.append((e, -1, i))
    ev.sort()
    active = set()
    last = t0
    conc = collections.Counter()
    alone = collections.Counter()
    shared = collections.Counter()
    pair = collections.Counter()
    for t, d, i in ev:
        dt = t - last
        if dt > 0:
            conc[min(len(active), 3)] += dt
            names = sorted(rows[j][2] for j in active)
            for j in active:
                (alone if len(active) == 1 else shared)[rows[j][2]] += dt
            if len(active) == 2:
                pair[" + ".join(names)] += dt
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    span = t1 - t0
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, n in rows:
        tot[n] += e - s
        cnt[n] += 1
    res = {
        "trace": os.path.relpath(f),
        "window_ms": span / 1e6,
        "k1_launches_in_window": len(k1) - 3,
        "time_with_kernels_in_flight_ms": {str(k if k < 3 else "3+"): conc[k] / 1e6 for k in (0, 1, 2, 3)},
        "per_kernel": {n: {"launches": cnt[n], "sum_ms": tot[n] / 1e6, "alone_ms": alone[n] / 1e6,
                           "beside_another_ms": shared[n] / 1e6}
                       for n in sorted(tot, key=lambda k: -tot[k])},
        "two_kernel_pairs_ms": {k: v / 1e6 for k, v in pair.most_common(8)},
    }
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
