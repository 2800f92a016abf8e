#!/usr/bin/env python3
"""Phase split of hs_match_kernel's reference-order Gauss-Newton step, measured by the `mclk` diagnostic
build (tools/build_diag.py mclk): the chain wave's s_memtime cycles per phase (step start -> chain start,
the chain, chain end -> next step), summed over all streams of K steps (hs_get_diag_stamps).  W warm-up steps build the maps with forced updates, then the map-update gate is set out of reach,
so the timed steps run the match only (the update kernel exits at once and leaves the counters alone).
GPU only:  SLAM2D_LIB=.../libslam2d_mclk.so python tools/clk_match.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "creating-2d-laser-slam-from-scratch_amd", "python"))
from slam2d import synth  # noqa: E402
from slam2d.hector import HectorFleet, HsLaser  # noqa: E402

B, T, W = int(os.environ.get("CLK_STREAMS", 3840)), 8, 4
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
fleet.set_thresholds(1e9, 1e9)
fleet.diag_stamps(reset=True)
t0 = time.perf_counter()
fleet.run_ranges_device(T - W, d_rng[W].data_ptr(), nb, B * nb, hip_stream=hs)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
st = fleet.diag_stamps(reset=True)
n = B * 14 * (T - W)  # Gauss-Newton steps timed (3 levels: 4 + 4 + 6 per match)
nbig = max(int(st[3]), 1)  # of them with >= 512 neighbourhood misses (a level's first step)
print(f"{T - W} match-only steps of {B} streams in {dt * 1e3:.2f} ms ({dt * 1e3 / (T - W):.3f} ms per step); {n} GN steps")
for name, v in (("pre-chain (transform, gathers, conversions, chunk 0)", st[0]), ("chain (1081 adds x 9 lanes)", st[1]),
                ("tail (solve, broadcast, barrier)", st[2])):
    print(f"{name:55s} {v / n:9.0f} cycles per GN step")
print(f"chain cycles per term: {st[1] / n / 1081:.2f}")
# point wave 0, lane 0 (same GN steps): start -> parked (transform + gathers returned + parking stores),
# parked -> the shared conversion's two barriers passed, -> chunk 0's terms stored and its barrier passed
for name, v in (("point wave: transform + gathers + parking", st[4]), ("point wave: shared conversion", st[5]),
                ("point wave: chunk 0 terms", st[6])):
    print(f"{name:55s} {v / n:9.0f} cycles per GN step")
if os.environ.get("CLK_BAR") == "1":  # the mclkbar build: stamp 3 = chain-wave cycles inside chunk barriers
    print(f"{'chain: inside its chunk barriers (chunks 1..)':55s} {st[3] / n:9.0f} cycles per GN step")
else:
    print(f"steps with >= 512 misses: {nbig} ({nbig / n:.3f} of all); their shared conversion {st[7] / nbig:.0f} cycles, "
          f"the other steps' {(st[5] - st[7]) / max(n - nbig, 1):.0f}")
fleet.close()
