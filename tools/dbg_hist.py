import ctypes, sys, numpy as np
sys.path.insert(0, '.')
import photohive_dsp_amd as phd
from photohive_dsp_amd import lib as L, synth
from photohive_dsp_amd.core import make_config
import torch
from tests.test_gpu_parity import _trace
from tests.conftest import golden_case
img = synth.make('vblur', 480, 640, 4)
g = golden_case('vblur_480x640')
cfg = make_config()
t = torch.from_numpy(img).cuda()
gid = torch.empty(480*640, dtype=torch.int32, device='cuda')
L.lib.phd_debug_hsv_groups_device(t.data_ptr(), 480*640, ctypes.byref(cfg), gid.data_ptr(), None)
gid = gid.cpu().numpy()
h_dbg = np.bincount(gid, minlength=112)
h_k1, par, kept = _trace(img)
print('dbg==golden', np.array_equal(h_dbg, g['hist']), 'k1==golden', np.array_equal(h_k1, g['hist']))
d = np.nonzero(h_k1 != g['hist'])[0]
print('groups differing', d, h_k1[d], g['hist'][d], h_dbg[d])
# per chunk
for c in range(0, 480*640, 16384):
    sub = np.bincount(gid[c:c+16384], minlength=112)[d]
    print(c//16384, sub)
