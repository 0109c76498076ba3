"""Child process of tests/test_gpu_round6.py (not collected: no test_ prefix).
Runs a two-lane device batch of 16 4000x3000 images (uniform / structured
alternating) in a fresh process; mode "explicit" then calls phd_shutdown, runs
the batch again on fresh contexts and compares every report field; mode
"atexit" leaves the teardown to the library's atexit handler.  Prints one
JSON line; the parent asserts exit status 0."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.lanes_hwq_child import digest  # noqa: E402


def main():
    mode = sys.argv[1]
    n, h, w = 16, 3000, 4000
    import torch
    torch.cuda.set_device(0)
    import photohive_dsp_amd as phd
    from photohive_dsp_amd.lib import lib
    nb = h * w * 3
    t = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    flat = t.view(-1)
    for i in range(n):
        if i % 2 == 0:
            assert lib.phd_fill_uniform_device(flat[i * nb:].data_ptr(), nb, 9100 + i, None) == 0
        else:
            assert lib.phd_fill_structured_device(flat[i * nb:].data_ptr(), h, w, 9100 + i, 15, 1, None) == 0
    torch.cuda.synchronize()
    lib.phd_set_lanes(2)
    first = [digest(r) for r in phd.report_device(t)]
    threads = lib.phd_debug_library_threads(0)
    out = {"mode": mode, "images": len(first), "threads_after_batch": threads}
    if mode == "explicit":
        lib.phd_shutdown()
        out["threads_after_shutdown"] = lib.phd_debug_library_threads(0)
        again = [digest(r) for r in phd.report_device(t)]
        same = 0
        for a, b in zip(first, again):
            same += all(a[f] == b[f] for f in a if f not in ("sbar", "hsv"))
        out["identical_after_restart"] = same
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
