"""How many run starts each thread of the column walk meets (fft_ct.hip,
walk_runs): the polar bin of every half-spectrum element (as
orc_blur_bin_of, oracle/phd_oracle.c, with numpy's atan2 / sqrt -- close
enough for counting), then per column and thread (E rows of T) the rows > 0
where the bin changes, and per wave the busiest lane.
  python tools/col_run_stats.py [H W nr na T]"""
import sys
import numpy as np

H, W, nr, na, T = (int(a) for a in sys.argv[1:6]) if len(sys.argv) > 5 else (3000, 4000, 40, 72, 256)
wf = W // 2 + 1
u = np.arange(H)[:, None]
x = np.arange(wf)[None, :]
top = u < H // 2
y = np.where(top, u, H - 1 - u)
phi = np.where(top, -np.arctan2(y, x), np.arctan2(y, x))
pb = ((phi + np.float32(np.pi) * 0.5) / np.float32(np.pi) * (na - 1)).astype(int)
rbss = float((wf * wf + H * H // 4) // (nr * nr))
rb = np.floor(np.sqrt((x * x + y * y) / rbss)).astype(int)
rb[rb == nr] -= 1
m = pb * nr + rb
ch = np.zeros_like(m, dtype=bool)
ch[1:] = m[1:] != m[:-1]
E = (H + T - 1) // T
pad = np.zeros((E * T, wf), bool)
pad[:H] = ch
pad = pad.reshape(T, E, wf)
pad[:, 0, :] = False                      # a start at the thread's first row is its segment's run
k = pad.sum(1)                            # [T, wf]
print(f"{H}x{W}, {na}x{nr} bins, T={T}, E={E}")
print("lanes by run starts met (0, 1, 2, ...):", np.round(np.bincount(k.ravel())[:6] / k.size, 4).tolist())
kw = k.reshape(T // 64, 64, wf).max(1)
print("waves whose busiest lane meets <= 2:", round(float((kw <= 2).mean()), 4))
