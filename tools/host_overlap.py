"""Host-buffer pipeline trace (run ON the GPU box):

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/hov -o hov -- \
        python tools/host_overlap.py run
    python tools/host_overlap.py analyse gpurun_out/hov

`run`: 64 pageable 3000x4000 RGB8 host buffers through phd_report_batch_u8
(one warm-up batch, then one traced batch).  `analyse`: from the kernel and
memory-copy traces of the LAST batch, the time the H2D copies and the kernels
are busy, how much of it overlaps, and the wall span, written to
gpurun_out/host_overlap.json."""
import csv
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(n=64, h=3000, w=4000, batches=2):
    import numpy as np
    import torch
    torch.cuda.set_device(0)
    from photohive_dsp_amd.lib import lib, last_error
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    nb = h * w * 3
    t = torch.empty(nb, dtype=torch.uint8, device="cuda")
    imgs = []
    for i in range(n):
        assert lib.phd_fill_uniform_device(t.data_ptr(), nb, 9000 + i, None) == 0
        imgs.append(t.cpu().numpy().copy())
    del t
    torch.cuda.synchronize()
    cfg = make_config()
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in imgs])
    hs = (ctypes.c_int * n)(*([h] * n))
    ws = (ctypes.c_int * n)(*([w] * n))
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()
    rates = []
    for k in range(batches):
        if k == 1:
            time.sleep(0.05)          # a gap in the trace marks the traced batch
        t0 = time.perf_counter()
        if lib.phd_report_batch_u8(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st) != 0:
            raise RuntimeError(last_error())
        dt = time.perf_counter() - t0
        for i in range(n):
            lib.free_full_report(ctypes.byref(outs[i]))
        print(f"batch {k}: {n} images in {1000 * dt:.1f} ms = {n / dt:.0f} images/s")
        rates.append(n / dt)
    if batches > 2:
        print(f"median of batches 1..: {sorted(rates[1:])[len(rates[1:]) // 2]:.0f} images/s")


def _intervals(path, kind):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if kind == "copy" and "HOST_TO_DEVICE" not in r.get("Direction", ""):
                continue
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def _union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _length(iv):
    return sum(b - a for a, b in iv)


def _intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append((a, b))
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def analyse(d):
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    cf = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    kern, copy = _intervals(kf, "kernel"), _intervals(cf, "copy")
    allv = sorted(kern + copy)
    # the traced batch: everything after the largest idle gap
    gaps = [(allv[i + 1][0] - max(b for _, b in allv[:i + 1]), i) for i in range(len(allv) - 1)]
    start = allv[max(gaps)[1] + 1][0]
    kern = _union([x for x in kern if x[0] >= start])
    copy = _union([x for x in copy if x[0] >= start])
    span = max(kern[-1][1], copy[-1][1]) - min(kern[0][0], copy[0][0])
    both = _length(_intersect(kern, copy))
    res = {"batch": "64 x 3000x4000 pageable host buffers, phd_report_batch_u8 (the second, traced batch)",
           "wall_span_ms": round(span / 1e6, 3), "h2d_busy_ms": round(_length(copy) / 1e6, 3),
           "kernels_busy_ms": round(_length(kern) / 1e6, 3), "overlap_ms": round(both / 1e6, 3),
           "h2d_busy_frac_of_span": round(_length(copy) / span, 3),
           "kernel_time_under_copies_frac": round(both / max(1, _length(kern)), 3)}
    print(json.dumps(res, indent=1))
    with open(os.path.join(ROOT, "gpurun_out", "host_overlap.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(batches=int(sys.argv[2]) if len(sys.argv) > 2 else 2)
    else:
        analyse(sys.argv[2])
