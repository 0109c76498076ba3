"""The C restatement (oracle/phd_oracle.c) under AddressSanitizer and
UndefinedBehaviorSanitizer: oracle/Makefile `sanitize` builds
oracle/sanitize_main.c with it and runs every entry point over synthetic
images (odd sizes, fine grids, overflowing linked lists, downsampling, crops,
a naive-DFT blur profile).  Any sanitizer report fails the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_clean_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_san", "oracle_san")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize OK" in r.stdout
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
