"""GPU idle time per bench step from a rocprofv3 kernel trace (run anywhere):

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sg -o sg -- python bench.py --no-configs ...
    python tools/step_gaps.py gpurun_out/sg

A step starts at a K1 (k_k1t) dispatch; prints each step's span, the time no
kernel or copy runs, and the gaps above 3 us with the dispatch that follows."""
import csv
import glob
import os
import sys


def main(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48])
                  for r in csv.DictReader(open(f)))
    k1 = [i for i, r in enumerate(rows) if "k_k1t" in r[2]]
    for a, b in zip(k1[-4:-1], k1[-3:]):
        seg = rows[a:b]
        t0, t1 = seg[0][0], rows[b][0]
        busy, (cs, ce) = 0, seg[0][:2]
        gaps = []
        for s, e, n in seg[1:] + [rows[b]]:
            if s > ce:
                busy += ce - cs
                if s - ce > 3000:
                    gaps.append(f"{(s - ce) / 1e3:.1f} us before {n.split('(')[0][-30:]}")
                cs, ce = s, e
            else:
                ce = max(ce, e)
        print(f"step {(t1 - t0) / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms: " + "; ".join(gaps))


if __name__ == "__main__":
    main(sys.argv[1])
