"""Child process of tests/test_gpu_round5.py::test_two_lanes_eight_hw_queues_fresh_process
(not collected: no test_ prefix).  GPU_MAX_HW_QUEUES is set by the parent
before this process starts, so HIP initialises with it.  Runs the same device
batch of 4000x3000 images on two library lanes (three times) and on one, and
prints one JSON line: which fields differ between the lane counts."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def digest(r):
    st = r.rgb_stats
    return {"stats": [st.Br, st.Bg, st.Bb, st.Cr, st.Cg, st.Cb],
            "sbar": r.average_saturation,
            "ids": list(r.color_palette.group_ids),
            "pct": list(r.color_palette.quantities),
            "hsv": np.array(r.color_palette.hsv, dtype=np.float64).ravel().tolist(),
            "bins": np.array(r.blur_profile.bins, dtype=np.float64).ravel().tolist(),
            "vec": [(v.angle, float(v.magnitude)) for v in r.blur_vectors]}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    h, w = 3000, 4000
    import torch
    torch.cuda.set_device(0)
    import photohive_dsp_amd as phd
    from photohive_dsp_amd.lib import lib
    nb = h * w * 3
    t = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    flat = t.view(-1)
    for i in range(n):
        # uniform and structured (hblur) images alternate: both palette tails run
        if i % 2 == 0:
            assert lib.phd_fill_uniform_device(flat[i * nb:].data_ptr(), nb, 7000 + i, None) == 0
        else:
            assert lib.phd_fill_structured_device(flat[i * nb:].data_ptr(), h, w, 7000 + i, 15, 1, None) == 0
    torch.cuda.synchronize()
    prev = lib.phd_set_lanes(2)
    runs2 = [[digest(r) for r in phd.report_device(t)] for _ in range(3)]
    lib.phd_set_lanes(1)
    one = [digest(r) for r in phd.report_device(t)]
    lib.phd_set_lanes(prev)
    diffs = []
    for k, run in enumerate(runs2):
        for i, (a, b) in enumerate(zip(one, run)):
            for f in a:
                if f == "sbar":
                    if abs(a[f] - b[f]) > 1e-12 * abs(a[f]):
                        diffs.append((k, i, f))
                elif f == "hsv":
                    # the palette's h / s sums are fp64 atomics (LDS and global):
                    # their order, and so the last bits, differ run to run
                    if len(a[f]) != len(b[f]) or not np.allclose(a[f], b[f], rtol=1e-12, atol=0):
                        diffs.append((k, i, f))
                elif a[f] != b[f]:
                    diffs.append((k, i, f))
    print(json.dumps({"hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"), "images": n, "two_lane_runs": len(runs2),
                      "diffs": diffs[:20], "n_diffs": len(diffs)}), flush=True)


if __name__ == "__main__":
    main()
