"""The CPU oracle (oracle/phd_oracle.c) against the reference's golden vectors.

The fixtures were produced by the reference's own C (tests/golden/make_golden.py);
passing here is what pins the oracle that the GPU parity tests rely on.
"""
import hashlib

import numpy as np
import pytest

import os

from tests.conftest import BIG_PIXELS, golden_case, golden_image, golden_manifest

CASES = [c for c in golden_manifest()["cases"]]
# the 120 MP cases take ~75 s of oracle time: checked when PHD_ORACLE_BIG=1
# (passed when the fixtures were made); the GPU suite compares against them
# at every run
BIG = {c["name"] for c in CASES if c["height"] * c["width"] >= BIG_PIXELS}


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_fixture(case):
    from oracle import oracle as orc
    if case["name"] in BIG and not os.environ.get("PHD_ORACLE_BIG"):
        pytest.skip("120 MP oracle run: set PHD_ORACLE_BIG=1")

    g = golden_case(case["name"])
    img = golden_image(case)
    assert hashlib.sha256(img.tobytes()).digest() == g["image_sha"].tobytes(), "generator drifted"
    r = orc.report(img, crops=case["crops"], **case["config"])
    # integer / index work: bit-exact
    np.testing.assert_array_equal(r.hist, g["hist"])
    np.testing.assert_array_equal(r.valid_parents, g["valid_parents"])
    np.testing.assert_array_equal(r.kept, g["kept"])
    np.testing.assert_array_equal(r.bin_counts, g["bin_counts"])
    np.testing.assert_array_equal(r.blur_angles, g["blur_angles"])
    np.testing.assert_array_equal(r.blur_mags, g["blur_mags"])
    assert r.angle_bin_size == int(g["angle_bin_size"])
    assert r.radius_bin_size == int(g["radius_bin_size"])
    # the restatement keeps the reference's evaluation order: floats are exact too
    np.testing.assert_array_equal(r.stats, g["stats"])
    assert r.average_saturation == float(g["average_saturation"])
    np.testing.assert_array_equal(r.palette_pct, g["palette_pct"])
    np.testing.assert_array_equal(r.palette_hsv, g["palette_hsv"])
    # DFT: pocketfft via numpy on both sides; keep a tolerance in case scipy is used
    np.testing.assert_allclose(r.bins, g["bins"], rtol=1e-12, atol=1e-15)
    if "sharpness" in g:
        np.testing.assert_array_equal(r.sharpness, g["sharpness"])


def test_oracle_error_shapes(manifest):
    from oracle import oracle as orc

    for e in manifest["errors"]:
        assert bool(orc.lib().orc_precheck(e["height"], e["width"])) == e["rejected"], e


def test_newton_int_sqrt_overshoots():
    """newton_int_sqrt (utilities.c:43-52) is not floor(sqrt): it can overshoot by one."""
    from oracle import oracle as orc

    vals = np.arange(0, 2000, 0.37)
    got = np.array([orc.lib().orc_newton_int_sqrt(float(v)) for v in vals])
    assert np.all(got >= np.floor(np.sqrt(vals)))
    assert np.any(got > np.floor(np.sqrt(vals)))
