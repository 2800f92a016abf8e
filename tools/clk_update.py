#!/usr/bin/env python3
"""Phase split of hs_update_kernel's tile loop, measured by the `clk` diagnostic build
(tools/build_diag.py clk): per-wave clock64() cycles of raster / pending apply / barrier wait / mark read,
summed over all waves of K north-star steps.  GPU only:  SLAM2D_LIB=.../libslam2d_clk.so python tools/clk_update.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "creating-2d-laser-slam-from-scratch_amd", "python"))
from slam2d import synth  # noqa: E402
from slam2d.hector import HectorFleet, HsLaser  # noqa: E402

B, T, W = int(os.environ.get("CLK_STREAMS", 2048)), 8, 3
S = synth.make_streams(B, T, seed=12345)
d_rng = torch.from_numpy(np.ascontiguousarray(S.ranges.transpose(1, 0, 2))).cuda()
nb = S.ranges.shape[2]
ang = synth.beam_angles(nb)
fleet = HectorFleet(B, 0.05, 2048, (0.5, 0.5), 3, max_points=1081)
fleet.set_update_factors(0.4, 0.9)
fleet.set_thresholds(-1.0, -1.0)
fleet.set_laser(HsLaser.defaults(nb, float(ang[0]), float(ang[1] - ang[0])), unit_vectors=np.stack([np.cos(ang), np.sin(ang)], 1))
hs = torch.cuda.current_stream().cuda_stream
fleet.run_ranges_device(W, d_rng[0].data_ptr(), nb, B * nb, hip_stream=hs)
torch.cuda.synchronize()
fleet.counters(reset=True)
fleet.run_ranges_device(T - W, d_rng[W].data_ptr(), nb, B * nb, hip_stream=hs)
torch.cuda.synchronize()
c = fleet.counters(reset=True)
ph = {"raster": c["gn_points"], "pending apply": c["updates"], "barrier wait": c["steps"], "mark read": c["touched"]}
tot = sum(ph.values())
for k, v in ph.items():
    print(f"{k:14s} {v / tot:6.3f}  ({v:.3e} wave-cycles)")
fleet.close()
