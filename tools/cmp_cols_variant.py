"""Compare the blur bins of two column-pass variants on the same images
(PHD_CT_COLS_VARIANT is read once per process, so each runs in a child):
    python tools/cmp_cols_variant.py A B [--H 3000 --W 4000]"""
import argparse
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import ctypes, sys
sys.path.insert(0, %(root)r)
import numpy as np, torch
torch.cuda.set_device(0)
from photohive_dsp_amd import synth
from photohive_dsp_amd.core import blur_profiles_device
imgs = [synth.make(k, %(H)d, %(W)d, s) for k, s in (("uniform", 1), ("structured", 2), ("dominant", 3))]
t = torch.from_numpy(np.stack(imgs)).cuda()
bins, vecs = blur_profiles_device(t)
np.save(%(out)r, np.asarray(bins))
"""


def main():
    p = argparse.ArgumentParser()
    p.add_argument("a")
    p.add_argument("b")
    p.add_argument("--H", type=int, default=3000)
    p.add_argument("--W", type=int, default=4000)
    a = p.parse_args()
    res = []
    for v in (a.a, a.b):
        out = f"/tmp/cmpv_{v}.npy"
        env = dict(os.environ, PHD_CT_COLS_VARIANT=v)
        r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "H": a.H, "W": a.W, "out": out}], env=env,
                           capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(r.stderr[-2000:])
            return 1
        res.append(np.load(out))
    x, y = res
    d = np.abs(x - y)
    rel = d / np.maximum(np.abs(y), 1e-300)
    print(f"variant {a.a} vs {a.b}: max abs {d.max():.3e} max rel {rel[y != 0].max() if (y != 0).any() else 0:.3e} "
          f"bit-identical {np.array_equal(x, y)}")
    for i in range(x.shape[0]):
        ratio = x[i][y[i] != 0] / y[i][y[i] != 0]
        print(f"  image {i}: ratio min {ratio.min():.15f} max {ratio.max():.15f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
