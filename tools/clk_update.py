#!/usr/bin/env python3
"""Phase split of hs_update_kernel's tile loop, measured by the `uclk` diagnostic build
(tools/build_diag.py uclk): per-wave s_memtime cycles of raster (ballot + clip + walk), the load / store wait
(vmcnt), the apply, the tile barrier and the mark read, summed over all waves of the north-star steps.
GPU only:
    SLAM2D_LIB=.../lib/ab/libslam2d_uclk.so python3 tools/clk_update.py [streams]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "creating-2d-laser-slam-from-scratch_amd", "python"))
from slam2d import synth  # noqa: E402
from slam2d.hector import HectorFleet, HsLaser  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 3840
T, W = 8, 3
S = synth.make_streams(B, T, seed=12345)
d_rng = torch.from_numpy(np.ascontiguousarray(S.ranges.transpose(1, 0, 2))).cuda()
nb = S.ranges.shape[2]
ang = synth.beam_angles(nb)
fleet = HectorFleet(B, 0.05, 2048, (0.5, 0.5), 3, max_points=1081)
fleet.set_update_factors(0.4, 0.9)
fleet.set_thresholds(-1.0, -1.0)
fleet.set_laser(HsLaser.defaults(nb, float(ang[0]), float(ang[1] - ang[0])),
                unit_vectors=np.stack([np.cos(ang), np.sin(ang)], 1))
hs = torch.cuda.current_stream().cuda_stream
fleet.run_ranges_device(W, d_rng[0].data_ptr(), nb, B * nb, hip_stream=hs)
torch.cuda.synchronize()
fleet.diag_stamps(reset=True)
fleet.run_ranges_device(T - W, d_rng[W].data_ptr(), nb, B * nb, hip_stream=hs)
torch.cuda.synchronize()
st = fleet.diag_stamps(reset=True)
names = ["raster", "vm wait", "apply", "barrier", "mark read"]
tot = float(st[:5].sum())
out = {"streams": B, "steps": T - W, "waves": int(st[5]), "tile_iterations_per_wave": float(st[6]) / max(int(st[5]), 1),
       "cycles_per_wave": tot / max(int(st[5]), 1),
       "split": {n: round(float(v) / tot, 4) for n, v in zip(names, st[:5])}}
print(json.dumps(out))
fleet.close()
