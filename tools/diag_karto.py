"""Per-phase s_memtime stamps of kt_addscans_kernel (diagnostic lib built with -DKT_DIAG_STAMPS):
SLAM2D_LIB=.../libslam2d_stamps.so python tools/diag_karto.py"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "creating-2d-laser-slam-from-scratch_amd", "python"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import torch  # noqa: E402
from slam2d import karto, _lib  # noqa: E402

M = int(os.environ.get("M", "512"))
lz, p, ranges, poses, query, beg, idx, NB, pen, ref = bench.karto_setup("karto", M, 777)
S = ranges.shape[0]
sm = karto.ScanMatcher(lz, p, max_matches=M, max_scans=S, max_base=NB)
dev = torch.device("cuda", 0)
d_r, d_p = torch.from_numpy(ranges).to(dev), torch.from_numpy(poses).to(dev)
d_q, d_b, d_i = (torch.from_numpy(a).to(dev) for a in (query, beg, idx))
d_res = torch.zeros(M * C.sizeof(karto.KtResult), dtype=torch.uint8, device=dev)
for _ in range(3):
    sm.set_scans_device(0, S, d_r.data_ptr(), d_p.data_ptr())
    sm.match_batch_device(M, d_q.data_ptr(), d_b.data_ptr(), d_i.data_ptr(), d_res.data_ptr(), pen, ref)
torch.cuda.synchronize()
L = _lib.lib()
st = np.zeros(M * 8, np.uint64)
L.kt_diag_stamps(st.ctypes.data_as(C.c_void_p), M)
st = st.reshape(M, 8).astype(np.int64)
d = np.diff(st[:, :6], axis=1)
names = ["cells", "count+prefix", "scatter", "render+store", "rest passes"]
print("per-block cycles (s_memtime, 100 MHz):")
for k, nme in enumerate(names):
    print(f"  {nme:14s} mean {d[:, k].mean():10.0f}  max {d[:, k].max():10.0f}")
span = st[:, 5].max() - st[:, 0].min()
print("kernel span", span, "block total mean", (st[:, 5] - st[:, 0]).mean())
