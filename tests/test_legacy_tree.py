"""get_full_report_data's reports in the reference's allocation shape
(phd_legacy.cpp): every member is its own malloc, so a C
caller may free() members itself (src/interface.c:97-111 frees them one by
one) and free_full_report frees the rest.  CPU only: the tree comes from the
phd_debug_legacy_report hook, the same copy and release code the legacy entry
uses after its GPU pipeline."""
import ctypes
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_legacy_tree_members_freed_by_caller_under_asan(tmp_path):
    """phd_legacy.cpp and a C++ driver built with ASan + UBSan (LSan on):
    the caller free()s members, the library frees the rest -- no invalid
    free, no double free, no leak."""
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path / "legacy_asan"
    src = [os.path.join(ROOT, "tests", "native", "legacy_tree_asan.cpp"),
           os.path.join(ROOT, "photohive_dsp_amd", "csrc", "phd_legacy.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-o", str(exe)] + src, check=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "legacy tree OK" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "LeakSanitizer" not in r.stderr


def test_free_full_report_frees_a_legacy_tree_after_member_frees():
    """Through the shipped library's own free_full_report (ctypes, glibc's
    allocator checks): member free()s by the caller first, then the call."""
    from photohive_dsp_amd.lib import lib
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    rp = lib.phd_debug_legacy_report(5, 72, 40, 2)
    assert rp
    r = rp.contents
    assert r.color_palette.contents.N == 5
    assert r.blur_profile.contents.bins[71][39] == pytest.approx(71.039)
    assert r.sharpness.contents.sharpness[1] == 2.0
    for ptr in (r.color_palette.contents.averages, r.color_palette.contents.percentages):
        libc.free(ctypes.cast(ptr, ctypes.c_void_p))
    r.color_palette.contents.averages = None
    r.color_palette.contents.percentages = None
    libc.free(ctypes.cast(r.rgb_stats, ctypes.c_void_p))
    r.rgb_stats = None
    lib.free_full_report(ctypes.byref(rp))
    assert not rp                                   # *report = NULL, as src/interface.c:109
    lib.free_full_report(ctypes.byref(rp))          # NULL: ignored


def test_shutdown_joins_library_threads_and_process_exits_cleanly():
    """phd_shutdown stops and joins the lane worker and
    both host pools; the library can start them again afterwards, and the
    process exits 0 with the atexit teardown having nothing left to do.  (No
    GPU here: the contexts' HIP resources are the -m gpu test's,
    tests/test_gpu_round6.py.)"""
    import subprocess
    import sys
    code = ("from photohive_dsp_amd.lib import lib; "
            "a = lib.phd_debug_library_threads(1); lib.phd_shutdown(); b = lib.phd_debug_library_threads(0); "
            "c = lib.phd_debug_library_threads(1); lib.phd_shutdown(); lib.phd_shutdown(); "
            "d = lib.phd_debug_library_threads(0); print(a, b, c, d)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    a, b, c, d = map(int, r.stdout.split())
    assert a >= 1 and b == 0 and c == a and d == 0, (a, b, c, d)


def test_crash_maps_written_at_the_fault(tmp_path):
    """phd_install_crash_maps: a SIGSEGV writes /proc/self/maps at the fault
    (async-signal-safe) and the process still dies of the signal."""
    import signal
    import subprocess
    import sys
    pre = str(tmp_path / "crash")
    code = ("import ctypes, os; from photohive_dsp_amd.lib import lib; "
            f"assert lib.phd_install_crash_maps({pre!r}.encode()) == 0; "
            "ctypes.string_at(0)")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == -signal.SIGSEGV, (r.returncode, r.stderr[-2000:])
    maps = [p for p in os.listdir(tmp_path) if p.endswith(".maps")]
    assert len(maps) == 1, maps
    txt = (tmp_path / maps[0]).read_text()
    assert "libreport_data.so" in txt and "[stack]" in txt
