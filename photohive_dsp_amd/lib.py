"""Loads PhotoHive_DSP_lib/libreport_data.so (the MI355X build) -- same path
and argtypes as /root/reference/lib.py:20-37, plus the new entry points."""
import ctypes
import os

from .structures import (Blur_Profile, Blur_Vector, Crop_Boundaries, Full_Report_Data, Image_PGM, Image_RGB,
                         PhdConfig, RGB_Statistics)

def _preload_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64.so
    (SONAME libamdhip64.so.7) and its libraries NEED the unversioned name; if
    this library were loaded first it would bind /opt/rocm's copy and torch
    would then load a second runtime.  Loading torch's file first (without
    importing torch) makes both resolve to the same runtime."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)


def configure_hw_queues(n: int = 8) -> bool:
    """Opt-in: ask HIP for `n` hardware queues per device (GPU_MAX_HW_QUEUES).

    The two library lanes drive two HIP streams each beside HIP's own copy
    traffic; eight queues measured +2-4 % images/s over HIP's default four
    (DESIGN.md section 12), because unrelated streams then stop sharing a
    queue.  HIP reads the variable once, when its runtime initialises, so this
    only takes effect if called before the process's first HIP call (this
    package's or torch's).  Importing the package does NOT set it (it would
    change every HIP user in the process and leak into child processes);
    bench.py calls the equivalent itself (--hw-queues).  Returns True when
    the value was written, False when the process had already chosen one."""
    if os.environ.get("GPU_MAX_HW_QUEUES"):
        return False
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))
    return True


_preload_torch_hip_runtime()
directory = os.path.dirname(os.path.abspath(__file__))
lib_path = os.path.join(directory, "PhotoHive_DSP_lib/libreport_data.so")
if os.environ.get("PHD_LIB"):          # kernel-variant experiments (tools/); not for production
    lib_path = os.path.abspath(os.environ["PHD_LIB"])
if not os.path.exists(lib_path):
    raise ImportError(f"{lib_path} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "or `make -C photohive_dsp_amd/csrc` (there is no CPU fallback)")
lib = ctypes.CDLL(lib_path)

P = ctypes.POINTER
lib.get_full_report_data.restype = P(Full_Report_Data)
lib.get_full_report_data.argtypes = [
    P(Image_RGB), P(Crop_Boundaries),
    ctypes.c_int, ctypes.c_int, ctypes.c_int,
    ctypes.c_double, ctypes.c_double,
    ctypes.c_double, ctypes.c_int,
    ctypes.c_int, ctypes.c_int, ctypes.c_int,
    ctypes.c_float, ctypes.c_float,
    ctypes.c_double, ctypes.c_double, ctypes.c_int,
]
lib.get_blur_profile_visual.restype = P(Image_PGM)
lib.get_blur_profile_visual.argtypes = [P(Blur_Profile), ctypes.c_int, ctypes.c_int]

# new entry points (include/photohive_dsp.h)
lib.phd_config_default.argtypes = [P(PhdConfig)]
lib.phd_report_u8.restype = P(Full_Report_Data)
lib.phd_report_u8.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, P(PhdConfig),
                              P(Crop_Boundaries)]
lib.phd_report_batch_device.restype = ctypes.c_int
lib.phd_report_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_size_t, P(PhdConfig), P(P(Full_Report_Data)),
                                        P(ctypes.c_int), ctypes.c_void_p]
lib.phd_report_batch_device_mixed.restype = ctypes.c_int
lib.phd_report_batch_device_mixed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                              ctypes.POINTER(PhdConfig), ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p]
lib.phd_blur_batch_device.restype = ctypes.c_int
lib.phd_blur_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                      ctypes.POINTER(PhdConfig), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(Blur_Vector), ctypes.c_void_p]
lib.phd_hsv_stats_batch_device.restype = ctypes.c_int
lib.phd_hsv_stats_batch_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_size_t, P(RGB_Statistics), P(ctypes.c_double),
                                           ctypes.c_void_p]
lib.phd_report_batch_u8.restype = ctypes.c_int
lib.phd_report_batch_u8.argtypes = [P(ctypes.c_void_p), P(ctypes.c_int), P(ctypes.c_int), ctypes.c_int,
                                    P(PhdConfig), P(P(Full_Report_Data)), P(ctypes.c_int)]
lib.phd_palette_trace_device.restype = ctypes.c_int
lib.phd_palette_trace_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, P(PhdConfig),
                                         P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int), P(ctypes.c_int)]
lib.phd_blur_counts.restype = ctypes.c_int
lib.phd_blur_counts.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P(ctypes.c_longlong)]
lib.phd_fill_uniform_device.restype = ctypes.c_int
lib.phd_fill_uniform_device.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_void_p]
lib.phd_fill_structured_device.restype = ctypes.c_int
lib.phd_fill_structured_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p]
lib.phd_debug_hsv_groups_device.restype = ctypes.c_int
lib.phd_debug_hsv_groups_device.argtypes = [ctypes.c_void_p, ctypes.c_long, P(PhdConfig), ctypes.c_void_p,
                                            ctypes.c_void_p]
lib.phd_debug_k1_pixels.restype = ctypes.c_int
lib.phd_debug_k1_pixels.argtypes = [ctypes.c_void_p, ctypes.c_long, P(PhdConfig), ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]
lib.phd_profile_kernels.restype = ctypes.c_int
lib.phd_profile_kernels.argtypes = [ctypes.c_uint]
lib.phd_profile_read.restype = ctypes.c_int
lib.phd_profile_read.argtypes = [ctypes.c_int, P(ctypes.c_double), P(ctypes.c_long)]
lib.phd_set_lanes.restype = ctypes.c_int
lib.phd_set_lanes.argtypes = [ctypes.c_int]
KERNELS = ["hsv_stats", "fft_rows", "fft_cols", "palette_cutoffs", "palette_sums", "sharpness"]
lib.phd_debug_time_kernel.restype = ctypes.c_int
lib.phd_debug_time_kernel.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, P(PhdConfig),
                                      ctypes.c_int, ctypes.c_int, P(ctypes.c_double)]
lib.phd_debug_power_spectrum.restype = ctypes.c_int
lib.phd_debug_power_spectrum.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.phd_debug_log_mant.restype = ctypes.c_int
lib.phd_debug_log_mant.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
lib.phd_debug_col_runs_max.restype = ctypes.c_int
lib.phd_debug_col_runs_max.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
lib.phd_debug_column_form.restype = ctypes.c_int
lib.phd_debug_column_form.argtypes = [ctypes.c_int]
lib.phd_debug_gfft.restype = ctypes.c_int
lib.phd_debug_gfft.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_long]
lib.free_full_report.restype = None
lib.free_full_report.argtypes = [P(P(Full_Report_Data))]
lib.phd_free_reports.restype = None
lib.phd_free_reports.argtypes = [P(P(Full_Report_Data)), ctypes.c_int]
lib.phd_free_pgm.argtypes = [P(Image_PGM)]
# round-6 entry points, bound only when present: an A/B timing run may load an
# older build through PHD_LIB (tools/); the shipped library exports all of them
# (tests/test_abi.py checks every symbol of include/photohive_dsp.h)
for _name, _res, _args in (("phd_shutdown", None, []),
                           ("phd_install_crash_maps", ctypes.c_int, [ctypes.c_char_p]),
                           ("phd_debug_library_threads", ctypes.c_int, [ctypes.c_int]),
                           ("phd_debug_legacy_report", P(Full_Report_Data),
                            [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int])):
    try:
        _f = getattr(lib, _name)
    except AttributeError:
        continue
    _f.restype, _f.argtypes = _res, _args
lib.phd_last_error.restype = ctypes.c_char_p
lib.phd_device_info.restype = ctypes.c_int
lib.phd_device_info.argtypes = [ctypes.c_char_p, ctypes.c_int]
lib.phd_last_timings.restype = ctypes.c_int
lib.phd_last_timings.argtypes = [P(ctypes.c_double), ctypes.c_int]


def last_error() -> str:
    return (lib.phd_last_error() or b"").decode()
