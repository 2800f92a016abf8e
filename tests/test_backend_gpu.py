"""The MapRepHip drop-in's threading contract on the GPU (VERDICT r01 "make the Hector boundary real").

tests/cpp/hector_threads_test (built by __graft_entry__.build() from tests/cpp/) is a C++ host of the
C-ABI: a spin thread runs HectorSlamProcessor::update per scan through slam2d::HectorMapBackend
(include/slam2d/hector_map_backend.hpp, the Eigen-free core of include/slam2d/MapRepHip.h) while a
publish thread refreshes level 0 as getGridMap would (hector_slam.cc:254-317).  It checks that every
snapshot the publish thread saw equals the CPU oracle's map after the same number of updates, that the
update index only moves forward and moved while the spin thread ran, and that every pose is bit-exact.
"""
import os
import subprocess

import numpy as np
import pytest

from slam2d import synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "tests", "cpp", "build", "hector_threads_test")


@pytest.mark.parametrize("size,levels", [(512, 2), (1024, 3)])
def test_spin_and_publish_threads(gpu, tmp_path, size, levels):
    assert os.path.exists(BIN), "tests/cpp not built (python -c 'import __graft_entry__ as g; g.build()')"
    K = 60
    S = synth.make_streams(1, K, seed=2024)
    M = int(S.points.shape[2])
    with open(tmp_path / "scans.bin", "wb") as f:
        np.asarray([K, M], np.int32).tofile(f)
        S.counts[0].astype(np.int32).tofile(f)
        np.ascontiguousarray(S.points[0], np.float32).tofile(f)
    r = subprocess.run([BIN, str(tmp_path / "scans.bin"), str(size), str(levels)], capture_output=True, text=True,
                       timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert "errors 0" in r.stdout


SM_BIN = os.path.join(REPO, "tests", "cpp", "build", "sm_icp_test")


def test_sm_icp_dropin(gpu, tmp_path):
    """lesson3's sm_icp call site (plicp_odometry.cc:391) swapped for slam2d_sm_icp (include/slam2d/
    sm_icp_hip.h): LDPs built as LaserScanToLDP builds them (float theta, -1 readings outside
    (range_min, range_max)), the node's parameter values, per-pair first guesses; valid, iterations,
    nvalid and every bit of x / error equal oracle/plicp_oracle.c on the same LDP arrays (tests/cpp/
    sm_icp_test.cpp); an unsupported switch (do_compute_covariance) returns valid = 0."""
    assert os.path.exists(SM_BIN), "tests/cpp not built"
    K = 40
    rng = np.random.default_rng(11)
    gt = synth.trajectory(K + 1, 0.7)
    R = (synth.cast_ranges(gt, synth.world_segments()) + rng.normal(0, 0.01, (K + 1, synth.N_BEAMS))).astype(np.float32)
    R[:, ::97] = np.float32(35.0)          # beyond range_max: invalid
    guess = rng.normal(0, [0.02, 0.02, 0.01], (K, 3))
    with open(tmp_path / "pairs.bin", "wb") as f:
        np.asarray([K, synth.N_BEAMS], np.int32).tofile(f)
        np.asarray([synth.ANGLE_MIN, synth.ANGLE_INC, 0.1, 29.9], np.float32).tofile(f)
        R.tofile(f)
        guess.astype(np.float64).tofile(f)
    r = subprocess.run([SM_BIN, str(tmp_path / "pairs.bin")], capture_output=True, text=True, timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr
    assert f"pairs {K} valid {K} errors 0" in r.stdout
