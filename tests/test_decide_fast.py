"""The host palette decision's fast paths (block-list insertion scan for
custom_sort, src/utilities.c:132-153; nearest-order table for
group_irregular_pixels' parent search, src/color_quantization.c:342-479)
decide exactly as the swap-by-swap insertion sort and the all-parents search:
tools/decide_bench.cpp checks a histogram of a synthetic image plus 400
random ones (sparse, dense, tied, and counts large enough for
compare_quantities' INT_MIN side) per grid."""
import glob
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "*.o")))
    if not objs:
        pytest.skip("native objects not built (run __graft_entry__.build())")
    out = str(tmp_path_factory.mktemp("db") / "decide_bench")
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    os.path.join(ROOT, "tools", "decide_bench.cpp"), *objs, "-L/opt/rocm/lib", "-lamdhip64",
                    "-o", out], check=True)
    return out


@pytest.mark.parametrize("grid", [(18, 2, 3), (36, 4, 5), (40, 6, 8), (360, 1, 1)])
def test_fast_decision_matches_insertion_sort(harness, grid, tmp_path):
    from oracle import oracle as orc
    from photohive_dsp_amd import synth
    h, s, v = grid
    img = synth.make("structured", 256, 256, 9)
    g = np.asarray(orc.group_ids(img, h_partitions=h, s_partitions=s, v_partitions=v)).ravel()
    hist = np.bincount(g, minlength=h * s * v + v + 1).astype(np.uint32)
    f = tmp_path / "hist.bin"
    hist.tofile(f)
    r = subprocess.run([harness, str(f), str(h), str(s), str(v), "3"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "histograms identical" in r.stdout
