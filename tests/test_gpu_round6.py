"""Round-6 GPU tests: the library's explicit teardown (phd_shutdown, also run
by its atexit handler) in fresh processes after two-lane batches, and the
legacy entry's reports in the reference's allocation shape (members freed by
the caller with free())."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.test_gpu_parity import _phd

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _child(mode):
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")      # the bench's configuration
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "shutdown_child.py"), mode],
                       env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert "SIGSEGV" not in r.stderr and "Segmentation" not in r.stderr, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_two_lane_batch_then_exit_status_zero():
    """A two-lane batch, then process exit with the teardown left to the
    library's atexit handler (threads joined, HIP resources released before
    HIP's own finalizers): exit status 0."""
    d = _child("atexit")
    assert d["images"] == 16 and d["threads_after_batch"] >= 1


def test_explicit_shutdown_then_fresh_contexts_identical():
    """phd_shutdown joins every library thread and frees every context; the
    next batch builds fresh contexts and gives identical reports."""
    d = _child("explicit")
    assert d["threads_after_shutdown"] == 0
    assert d["identical_after_restart"] == 16


def test_legacy_entry_members_freed_by_caller():
    """get_full_report_data's report: every member a separate malloc
    (src/interface.c:97-111), so the caller may free() members itself; the
    values equal the u8 entry's report."""
    phd, L, _ = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.utils import pil_image_to_image_rgb
    from PIL import Image
    img = synth.make("structured", 384, 512, 77)
    pil = Image.fromarray(img)                       # owns the planes (utils.py keeps them on it)
    im = pil_image_to_image_rgb(pil)
    ptr = L.lib.get_full_report_data(ctypes.byref(im), None, 18, 2, 3, 0.1, 0.1, 0.95, 1000, 1, 40, 72,
                                     0.1, 0.9, 1.20, 0.3, 2)
    assert ptr, L.last_error()
    ref = phd.get_report(img)
    r = ptr.contents
    cp = r.color_palette.contents
    assert cp.N == len(ref.color_palette.group_ids)
    assert [cp.averages[k].parent_id for k in range(cp.N)] == list(ref.color_palette.group_ids)
    bins = np.array([[r.blur_profile.contents.bins[a][q] for q in range(40)] for a in range(72)])
    np.testing.assert_allclose(bins, np.array(ref.blur_profile.bins), rtol=1e-12, atol=1e-14)
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    for a in range(72):                              # free_2d_array's rows, by the caller
        libc.free(ctypes.cast(r.blur_profile.contents.bins[a], ctypes.c_void_p))
        r.blur_profile.contents.bins[a] = None
    libc.free(ctypes.cast(cp.averages, ctypes.c_void_p))
    cp.averages = None
    libc.free(ctypes.cast(r.rgb_stats, ctypes.c_void_p))
    r.rgb_stats = None
    L.lib.free_full_report(ctypes.byref(ptr))
    assert not ptr
