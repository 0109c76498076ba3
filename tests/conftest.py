"""Shared pytest configuration.

`-m gpu` tests need a real MI355X and the built HIP library; everything else
runs on the CPU container.  The oracle (oracle/) is used here only as the
checker.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_case(name):
    with np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


BIG_PIXELS = 50_000_000          # the 120 MP fixtures: generated once per session
_big_images = {}


def golden_image(case):
    from photohive_dsp_amd import synth
    key = (case["kind"], case["height"], case["width"], case["seed"])
    if key in _big_images:
        return _big_images[key]
    img = synth.make(*key)
    if case["height"] * case["width"] >= BIG_PIXELS:
        _big_images[key] = img
    return img


@pytest.fixture(scope="session")
def manifest():
    return golden_manifest()
