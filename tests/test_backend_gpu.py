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
