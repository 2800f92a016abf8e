"""Host logic on the CPU: the DataContainer mirror, the synthetic scan generator, bench.py's
accounting helpers, and bench's rank aggregation over torch.distributed (gloo, world_size 2)."""
import ctypes as C
import json
import math
import os
import socket

import numpy as np
import pytest

import bench
from slam2d import synth
from slam2d.hector import DataContainer


# ----------------------------------------------------------------------------- DataContainer
def test_datacontainer_setfrom_scales_points_and_origo():
    """DataPointContainer::setFrom (scan/DataPointContainer.h:46-58): points and origo * factor."""
    d = DataContainer()
    d.add([2.0, 4.0])
    d.add([-1.0, 0.5])
    d.setOrigo([3.0, -2.0])
    e = DataContainer()
    e.setFrom(d, 0.5)
    assert e.getSize() == 2
    np.testing.assert_array_equal(e.getVecEntry(0), np.float32([1.0, 2.0]))
    np.testing.assert_array_equal(e.getOrigo(), np.float32([1.5, -1.0]))
    e.clear()
    assert e.getSize() == 0


def test_datacontainer_from_points_roundtrip():
    pts = np.random.default_rng(0).normal(size=(17, 2)).astype(np.float32)
    d = DataContainer.from_points(pts, (0.25, 0.5))
    np.testing.assert_array_equal(d.points(), pts)
    d.add([9.0, 9.0])
    assert d.getSize() == 18 and d.getVecEntry(17)[0] == 9.0


# ----------------------------------------------------------------------------- synthetic scans
def test_synth_deterministic_and_filtered():
    a = synth.make_streams(2, 6, seed=5)
    b = synth.make_streams(2, 6, seed=5)
    np.testing.assert_array_equal(a.points, b.points)
    np.testing.assert_array_equal(a.counts, b.counts)
    assert a.points.shape == (2, 6, synth.N_BEAMS, 2)
    assert (a.counts > 900).all() and (a.counts <= synth.N_BEAMS).all()
    # hector_slam.cc:336-353 filters: 0.2 m < d < 20 m (points are in map scale x20)
    for s in range(2):
        for k in range(6):
            p = a.points[s, k, : a.counts[s, k]] / 20.0
            d = np.hypot(p[:, 0], p[:, 1])
            assert d.min() > 0.2 and d.max() < 20.0


def test_synth_trajectory_step_bounds():
    """<= 0.1 m and <= 5 deg per scan."""
    S = synth.make_streams(3, 50, seed=9)
    for s in range(3):
        g = S.gt[s]
        step = np.hypot(np.diff(g[:, 0]), np.diff(g[:, 1]))
        dth = np.abs(np.angle(np.exp(1j * np.diff(g[:, 2]))))
        assert step.max() <= 0.1 + 1e-9 and dth.max() <= math.radians(5) + 1e-9


def test_synth_beam_geometry():
    a = synth.beam_angles()
    assert len(a) == 1081
    assert np.isclose(a[0], -3 * math.pi / 4, atol=1e-6)
    assert np.allclose(np.diff(a), math.radians(0.25), atol=1e-6)


# ----------------------------------------------------------------------------- bench accounting
def test_algorithmic_bytes_formula():
    """B_match = gn_points x 24 B, B_update = ΣL x 16 B, read-only = B_match + ΣL x 8."""
    ctr = {"gn_points": 1000, "cells": 5000, "rays": 70}
    ab = bench.algorithmic_bytes(ctr, 3)
    assert ab["match"] == 24000 and ab["update"] == 80000 and ab["total"] == 104000
    assert ab["read_only"] == 24000 + 40000 and ab["bin"] == 70 * 12


def test_kernel_symbol():
    kt = {"match": (1.0, 3), "bin": (0.0, 0), "update": (2.0, 3)}
    assert bench.kernel_symbol("update", kt) == "hs_update_kernel"
    kt["bin"] = (0.5, 3)
    assert bench.kernel_symbol("update", kt) == "hs_tile_kernel"
    assert bench.kernel_symbol("match", kt) == "hs_match_kernel"


def test_pmc_traffic_lookup(tmp_path, monkeypatch):
    """roofline.traffic is attached only from a summary of the SAME workload (config, streams, map-update
    semantics, summation order) and only when its launch time agrees with this run's (same build)."""
    p = tmp_path / "pmc.json"
    e = {"kernel": "hs_update_kernel<5>", "config": "northstar", "streams": 1024, "semantics": "forced", "order": 0,
         "avg_ns": 1000.0, "traffic_bytes_per_launch": 123, "source": "x"}
    p.write_text(json.dumps({"entries": [e]}))
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    w = {"config": "northstar", "streams": 1024, "semantics": "forced", "order": 0}
    got, why = bench.pmc_traffic("hs_update_kernel", w, 1100.0)
    assert got["traffic_bytes_per_launch"] == 123 and why == "x"
    for k, v in (("config", "c2"), ("streams", 2048), ("semantics", "reference"), ("order", 256), ("kernel_src", "x")):
        assert bench.pmc_traffic("hs_update_kernel", {**w, k: v}, 1000.0)[0] is None, k
    got, why = bench.pmc_traffic("hs_update_kernel", w, 2000.0)   # another build: refused
    assert got is None and "another build" in why


def test_committed_pmc_summary_is_consistent():
    """profiles/pmc_traffic.json: every entry points at a committed summary file."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(repo, "profiles", "pmc_traffic.json")) as f:
        d = json.load(f)
    for e in d["entries"]:
        assert os.path.exists(os.path.join(repo, e["source"])), e["source"]
        assert e["traffic_bytes_per_launch"] == int((2 * e["fetch_kb"] + e["write_kb"]) * 1024)


# ----------------------------------------------------------------------------- distributed (gloo)
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _agg_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t, u = bench.aggregate_over_ranks(1.0 + rank, 100.0 * (rank + 1), torch.device("cpu"))
    out[rank] = (t, u)
    dist.barrier()
    dist.destroy_process_group()


def test_rank_aggregation_gloo_world2():
    """bench.py: value = units of ALL ranks / the SLOWEST rank's time (barrier + max over ranks)."""
    import torch.multiprocessing as mp

    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_agg_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        assert res[r] == (2.0, 300.0)


def test_rank_aggregation_single_process():
    import torch

    assert bench.aggregate_over_ranks(0.5, 7.0, torch.device("cpu")) == (0.5, 7.0)


# ----------------------------------------------------------------------------- GMapping weight exchange (gloo)
def _weights_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from slam2d.gmapping import normalize_weights

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scores = torch.arange(rank * 3, rank * 3 + 3, dtype=torch.int32)   # this rank's particle shard
    w, neff = normalize_weights(scores)
    out[rank] = (w.tolist(), neff)
    dist.barrier()
    dist.destroy_process_group()


def test_particle_weight_allreduce_gloo_world2():
    """Sharded particles: one all-reduce gives weights identical to the single-process result."""
    import torch
    import torch.multiprocessing as mp

    from slam2d.gmapping import normalize_weights

    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_weights_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    w_all, neff_all = normalize_weights(torch.arange(0, 6, dtype=torch.int32))
    got = res[0][0] + res[1][0]
    np.testing.assert_allclose(got, w_all.tolist(), rtol=0, atol=0)
    assert abs(sum(got) - 1.0) < 1e-12
    assert res[0][1] == res[1][1] == neff_all


# ----------------------------------------------------------------------------- RCCL unique id over gloo
def _uid_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist

    from slam2d.gmapping import _UniqueId, exchange_unique_id, unique_id_bytes

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = _UniqueId()
    if rank == 0:  # an ncclUniqueId-like id: family 2 then NULs, a port, an address, random tail bytes
        raw = np.zeros(128, np.uint8)
        raw[:16] = [2, 0, 0x9C, 0x41, 127, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0]
        raw[100:128] = np.arange(1, 29, dtype=np.uint8)
        C.memmove(C.addressof(uid), raw.tobytes(), 128)

    def bcast(buf):  # the same callable bench.py hands RcclComm, on CPU tensors
        t = torch.from_numpy(np.ascontiguousarray(buf))
        dist.broadcast(t, 0)
        return t.numpy()

    got = exchange_unique_id(uid, world, rank, bcast)
    out[rank] = unique_id_bytes(got).tobytes()
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_unique_id_with_nul_bytes_gloo_world2():
    """RcclComm's id broadcast (exchange_unique_id) carries all 128 bytes of an id that holds NULs
    (a c_char field truncated it at the first NUL, so N > 1 could not start)."""
    import torch.multiprocessing as mp

    from slam2d.gmapping import _UniqueId, unique_id_bytes, unique_id_from_bytes

    world = 2
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_uid_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    assert len(res[0]) == len(res[1]) == 128
    assert res[0] == res[1]
    assert res[1][:2] == b"\x02\x00" and res[1][-1] == 28
    # round trip of the (de)serialisation itself
    raw = np.random.default_rng(3).integers(0, 256, 128).astype(np.uint8)
    raw[5] = 0
    assert unique_id_bytes(unique_id_from_bytes(raw)).tobytes() == raw.tobytes()
    with pytest.raises(Exception):
        unique_id_from_bytes(raw[:1])
    assert C.sizeof(_UniqueId) == 128


# ------------------------------------------------------------------ bench.py --gpus N launcher
def _bench_env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["PYTHONPATH"] = bench.REPO
    return env


def test_bench_gpus_n_launches_its_ranks():
    """`bench.py --gpus 2` with no external launcher starts 2 ranks itself (torch.distributed.run as a child
    process) and relays rank 0's one JSON line: n_gpus 2, the global batch is both ranks' units."""
    import subprocess
    import sys

    r = subprocess.run([sys.executable, os.path.join(bench.REPO, "bench.py"), "--gpus", "2", "--streams", "512",
                        "--cpu-cores", "2", "--launcher-selftest"], capture_output=True, text=True, timeout=300,
                       env=_bench_env())
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 1024, out
    # the CPU baseline is timed at N > 1 too (rank 0, the same block main() attaches)
    cpu = out["cpu_baseline"]
    assert cpu["cores"] == 1 and cpu["value"] > 0 and cpu["kind"] == "port", cpu
    assert cpu["all_cores"]["cores"] == 2 and cpu["all_cores"]["value"] > 0, cpu


def test_bench_world_size_mismatch_is_refused():
    """WORLD_SIZE set by a launcher but different from --gpus: exit non-zero instead of a mislabelled line."""
    import subprocess
    import sys

    env = _bench_env()
    env.update({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    r = subprocess.run([sys.executable, os.path.join(bench.REPO, "bench.py"), "--gpus", "1", "--launcher-selftest"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, (r.returncode, r.stderr[-500:])


def test_north_star_targets_block():
    """The bench line's targets block: each target with its value and pass/fail."""
    cpu = {"value": 1000.0, "kind": "port", "all_cores": {"value": 15000.0, "cores": 16}}
    roof = {"survey_8d_read_only_frac": 0.58, "read_only_frac_counters": 0.14, "read_share_of_counted": 0.387,
            "frac": 0.455, "traffic": 6650485317, "min_traffic_frac": 0.373}
    pose = {"max_abs_xy_m": 0.0, "max_abs_theta_rad": 0.0}
    t = bench.north_star_targets(1.4e6, cpu, roof, pose)
    assert t["x_cpu_1core"]["value"] == 1400.0 and t["x_cpu_1core"]["pass"]
    assert t["x_cpu_all_cores"]["cores"] == 16 and round(t["x_cpu_all_cores"]["value"], 2) == 93.33
    assert not t["x_cpu_all_cores"]["pass"]
    # counted bytes only: SURVEY 8d's touch model is not a target row (its rate can pass the HBM peak)
    assert "read_roofline_model" not in t
    assert t["hbm_roofline_counted"]["pass"] and t["hbm_roofline_distinct_cell_floor"]["value"] == 0.373
    assert not t["read_roofline_counted"]["pass"] and t["read_roofline_counted"]["bound"] == 0.387
    # without a PMC summary the counted row has no value (the floor fallback is not counted traffic)
    assert bench.north_star_targets(1.4e6, cpu, {"frac": 0.4, "traffic": None}, pose)["hbm_roofline_counted"]["value"] is None
    assert t["pose_error_m"]["pass"] and t["pose_error_rad"]["pass"]
    assert bench.north_star_targets(1.0, None, None, pose)["x_cpu_1core"]["pass"] is None


def test_diagnostic_build_anchors_apply():
    """tools/build_diag.py's pricing variants are textual patches of the kernel sources: every anchor must
    still occur exactly once, so a listed variant never fails at build time on the GPU box."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("build_diag", os.path.join(bench.REPO, "tools", "build_diag.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    assert m.check() == []
