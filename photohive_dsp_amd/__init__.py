"""PhotoHive_DSP for MI355X: drop-in get_report / Report / set_bounding_boxes
backed by hand-written HIP kernels (PhotoHive_DSP_lib/libreport_data.so)."""
from .core import Report, get_report, get_reports, report_device, set_bounding_boxes  # noqa: F401
from .lib import configure_hw_queues  # noqa: F401  (opt-in GPU_MAX_HW_QUEUES, before HIP starts)
