"""C-ABI surface (CPU): the library loads and exports every symbol
include/photohive_dsp.h declares; struct layouts match the reference's
ctypes binding; no GPU => loud failure, never a silent CPU fallback."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "photohive_dsp.h")
SO = os.path.join(ROOT, "photohive_dsp_amd", "PhotoHive_DSP_lib", "libreport_data.so")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\((?=[^;{]*\)\s*;)", src)
    keywords = {"if", "for", "while", "return", "sizeof"}
    return sorted({n for n in names if n not in keywords})


def test_header_declares_reference_entry_points():
    fns = declared_functions()
    for f in ("get_full_report_data", "free_full_report", "get_blur_profile_visual"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    assert os.path.exists(SO), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(SO)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_every_declared_function_has_ctypes_argtypes():
    """A pointer passed without argtypes is truncated to a C int by ctypes."""
    from photohive_dsp_amd.lib import lib
    missing = [f for f in declared_functions() if getattr(lib, f).argtypes is None and f != "phd_last_error"]
    assert not missing, missing


def test_struct_layouts_match_reference_binding():
    from photohive_dsp_amd import structures as S
    # x86-64 sizes of the reference structs (src/*.h)
    assert ctypes.sizeof(S.Pixel_HSV) == 32
    assert ctypes.sizeof(S.Image_RGB) == 32
    assert ctypes.sizeof(S.Image_PGM) == 16
    assert ctypes.sizeof(S.RGB_Statistics) == 48
    assert ctypes.sizeof(S.Crop_Boundaries) == 40
    assert ctypes.sizeof(S.Color_Palette) == 24
    assert ctypes.sizeof(S.Blur_Profile) == 24
    assert ctypes.sizeof(S.Blur_Vector) == 8
    assert ctypes.sizeof(S.Blur_Vector_Group) == 16
    assert ctypes.sizeof(S.Sharpnesses) == 16
    assert ctypes.sizeof(S.Full_Report_Data) == 48
    assert S.Full_Report_Data.average_saturation.offset == 32


def _our_layout():
    from photohive_dsp_amd import structures as S
    from tests.golden.make_struct_layout import layout
    return layout(S)


def test_every_field_offset_matches_reference_structures():
    """Every Structure of the reference's structures.py (its ctypes binding, the
    drop-in contract): same fields in the same order, same offsets, sizes and
    ctypes types.  Against the committed fixture (tests/golden/struct_layout.json,
    written from the reference by tests/golden/make_struct_layout.py)."""
    import json
    with open(os.path.join(os.path.dirname(__file__), "golden", "struct_layout.json")) as f:
        ref = json.load(f)
    ours = _our_layout()
    for name, want in ref.items():
        assert name in ours, f"{name} missing from photohive_dsp_amd/structures.py"
        assert ours[name] == want, (name, ours[name], want)


@pytest.mark.skipif(not os.path.exists("/root/reference/structures.py"),
                    reason="the reference tree exists only in the build container")
def test_field_offsets_match_live_reference_structures():
    """The same comparison against the reference's structures.py itself, read
    with `ast` (its `_fields_` literals; the file is never executed)."""
    from tests.golden.make_struct_layout import layout, parse_reference
    ref = layout(parse_reference())
    ours = _our_layout()
    for name, want in ref.items():
        assert ours.get(name) == want, (name, ours.get(name), want)


def test_config_defaults_match_get_report():
    from photohive_dsp_amd.lib import lib
    from photohive_dsp_amd.structures import PhdConfig
    from photohive_dsp_amd.core import make_config
    c = PhdConfig()
    lib.phd_config_default(ctypes.byref(c))
    d = make_config()
    for f, _ in PhdConfig._fields_:
        assert getattr(c, f) == getattr(d, f), f


def test_no_silent_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import photohive_dsp_amd as phd
    from photohive_dsp_amd.lib import last_error
    from photohive_dsp_amd import synth
    with pytest.raises(ValueError):
        phd.get_report(synth.uniform(400, 400, 1))
    assert "no HIP device" in last_error()


def test_reference_rejections_are_null_before_touching_gpu():
    """pre_compute_error_checks (src/utilities.c:64-87) paths return NULL."""
    import numpy as np
    import photohive_dsp_amd as phd
    from photohive_dsp_amd.lib import last_error
    for h, w in [(349, 350), (350, 349), (2001, 400), (400, 2001)]:
        with pytest.raises(ValueError):
            phd.get_report(np.zeros((h, w, 3), np.uint8))
        assert "350" in last_error() or "aspect" in last_error()


def test_lanes_default_is_two_and_phd_lanes_overrides():
    """The library's default is two lanes (phd_context.cpp lanes_setting);
    PHD_LANES=1 selects one (a fresh process each: the setting is read once)."""
    import subprocess
    import sys
    code = "from photohive_dsp_amd.lib import lib; print(lib.phd_set_lanes(0))"
    for env_val, want in ((None, 2), ("1", 1), ("2", 2)):
        env = {k: v for k, v in os.environ.items() if k != "PHD_LANES"}
        if env_val is not None:
            env["PHD_LANES"] = env_val
        out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                             timeout=120)
        assert out.returncode == 0, out.stderr
        assert int(out.stdout.strip().splitlines()[-1]) == want


def test_lanes_setting_and_batch_free_need_no_gpu():
    """phd_set_lanes clamps to 1..2 and lanes < 1 only query; phd_free_reports
    skips NULL entries and leaves every entry NULL (host-only calls)."""
    from photohive_dsp_amd.lib import lib
    from photohive_dsp_amd.structures import Full_Report_Data
    prev = lib.phd_set_lanes(0)
    assert prev in (1, 2)
    try:
        assert lib.phd_set_lanes(1) == prev
        assert lib.phd_set_lanes(7) == 1
        assert lib.phd_set_lanes(0) == 2
    finally:
        lib.phd_set_lanes(prev)
    outs = (ctypes.POINTER(Full_Report_Data) * 3)()
    lib.phd_free_reports(outs, 3)
    lib.phd_free_reports(None, 0)
    assert all(not outs[i] for i in range(3))


def test_gpurunignore_keeps_reference_builds_off_the_gpu_box():
    """reference sources and anything built from them
    never go to the GPU box.  oracle/Makefile writes the reference build into
    oracle/_ref/ (from REF_SRC) and the sanitizer build into oracle/_san/;
    both directories must be excluded from every gpurun snapshot."""
    ign = [l.strip() for l in open(os.path.join(ROOT, ".gpurunignore")) if l.strip() and not l.startswith("#")]
    mk = open(os.path.join(ROOT, "oracle", "Makefile")).read()
    outdirs = sorted(set(re.findall(r"\$\(HERE\)(_[a-z]+)/", mk)))
    assert "_ref" in outdirs and "_san" in outdirs, outdirs
    for d in outdirs:
        assert f"./oracle/{d}" in ign or f"oracle/{d}" in ign, (d, ign)


def test_free_full_report_ignores_foreign_pointers():
    """Reports are single pooled blocks (include/photohive_dsp.h): the library
    pools only blocks it handed out, so freeing a structure it did not
    allocate touches nothing around it and still clears the caller's pointer;
    a NULL report is a no-op (the reference would dereference it)."""
    from photohive_dsp_amd.lib import lib
    from photohive_dsp_amd.structures import Full_Report_Data
    guard = (ctypes.c_ubyte * 128)(*([0xAB] * 128))
    foreign = Full_Report_Data.from_buffer(guard, 32)
    p = ctypes.pointer(foreign)
    lib.free_full_report(ctypes.byref(p))
    assert not p                                    # *report = NULL
    assert all(b == 0xAB for b in guard)            # no header read or write around it
    null = ctypes.POINTER(Full_Report_Data)()
    lib.free_full_report(ctypes.byref(null))
    lib.phd_free_reports(None, 3)


def test_column_run_lists_fit_the_default_grid_only():
    """Host only: the compile-time column pass holds at most 256 run-list entries
    per spectrum column.  The default 72 x 40 grid at 4000x3000 and config 5's
    largest sizes fit; radius_partitions = 160 does not (that size takes the
    runtime-plan FFT, tests/test_gpu_round5.py)."""
    from photohive_dsp_amd.lib import lib
    for h, w in ((3000, 4000), (4000, 6000), (6000, 4000), (4000, 3000)):
        assert 0 < lib.phd_debug_col_runs_max(h, w, 40, 72) <= 256, (h, w)
    assert lib.phd_debug_col_runs_max(3000, 4000, 160, 72) > 256
    assert lib.phd_debug_col_runs_max(300, 4000, 40, 0) == -1
