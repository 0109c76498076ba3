"""Run single bench.py legs on the GPU (development helper):
    python tools/only.py config3 [config4 config5 headline ...]
Each leg prints its JSON object."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    legs = sys.argv[1:] or ["config3"]
    args = bench.parse(["--steps", os.environ.get("ONLY_STEPS", "30"), "--warmup", "4",
                        "--batch", os.environ.get("ONLY_BATCH", "64")])
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(args.hw_queues))   # as bench.main, before HIP starts
    import torch
    torch.cuda.set_device(0)
    import photohive_dsp_amd  # noqa: F401
    cx = bench.Ctx(args, 1, 0, "nccl")
    cx.lib.phd_set_lanes(int(os.environ.get("ONLY_LANES", "1")))
    for leg in legs:
        if leg in ("headline", "structured"):
            hl = bench.headline(cx, kind="hblur" if leg == "structured" else "uniform")
            m = hl["merged"]
            out = {"images_per_s": round(m["images"] / m["elapsed"], 1),
                   "ms_per_step": round(1000 * m["elapsed"] / hl["steps"], 3),
                   "dom": hl["dom"], "warm_us": {k: round(v["avg_us"], 2) for k, v in hl["warm"].items()},
                   "stages": {k: round(v, 3) for k, v in hl["stages"].items()}}
        elif leg == "config3":
            out = bench.config3(cx)
        elif leg == "config4":
            out = bench.config4(cx, args.config4_images)
        elif leg == "config5":
            out = bench.config5(cx, args.config5_images)
        elif leg == "single":
            out = bench.single_image(cx)
        else:
            raise SystemExit(f"unknown leg {leg}")
        print(leg, json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
