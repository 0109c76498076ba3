import ctypes, os, subprocess, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
from photohive_dsp_amd import synth
cfg = make_config(h_partitions=36, s_partitions=4, v_partitions=5)
tl = 36 * 4 * 5 + 5 + 1
for (h, w) in ((512, 512), (480, 640)):
    t = torch.empty(h * w * 3, dtype=torch.uint8, device="cuda")
    assert lib.phd_fill_uniform_device(t.data_ptr(), h * w * 3, 77, None) == 0
    hist = (ctypes.c_int * tl)(); par = (ctypes.c_int * tl)(); kept = (ctypes.c_int * tl)(); npar = ctypes.c_int()
    rc = lib.phd_palette_trace_device(t.data_ptr(), h, w, ctypes.byref(cfg), hist, par, kept, ctypes.byref(npar))
    a = np.array(hist[:], dtype=np.uint32)
    ref = synth.uniform(h, w, 77)
    print(h, w, "device image == synth.uniform:", np.array_equal(t.cpu().numpy().reshape(h, w, 3), ref), "npar", npar.value)
    a.tofile(f"/tmp/h{h}.bin")
    print(subprocess.run(["tools/_decide_bench", f"/tmp/h{h}.bin", "36", "4", "5", "50"], capture_output=True, text=True).stdout)
