#!/usr/bin/env python3
"""bench.py -- Hector scan-match + grid-update throughput on MI355X (BASELINE.json metric).

One step = one HectorSlamProcessor::update (match coarse->fine + log-odds raycast update of every
pyramid level) for each of B independent scan streams resident in HBM (inputs uploaded before the
timed region).  Benchmark mode forces a map update on every scan (thresholds < 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--streams B] [--config northstar|c2|c3|gmapping|plicp|karto|karto_loop]

Multi-GPU: launched by torch.distributed.run, one process per GPU; each rank runs its own B streams
(replicas only -- the Hector path has no cross-stream exchange), barrier + synchronize around the
timed region, max time over ranks, value = total scans of all ranks / that time.

Rank 0 prints ONE JSON line with value, roofline (dominant kernel, HIP-event timed inside the timed
region) and cpu_baseline (the CPU oracle, single core, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "creating-2d-laser-slam-from-scratch_amd")
sys.path.insert(0, os.path.join(PKG, "python"))

METRIC = "scans/sec (1081-beam) Hector match+grid-update @1 GPU; pose RMSE vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)

CONFIGS = {
    # hector_slam.launch defaults (hector_slam.cc:138-142): 2048^2, 3 levels -- the north-star grid.
    # 4608 streams x 52.5 MB pyramids (20-KB three-plane tiles) = 242 GB of HBM: three whole rounds of
    # the match at 6 workgroups per CU (round 6; 3840 = three rounds at 5 per CU before).  One lease
    # (profiles/r06/ab_r06k_match6_vs_prev.md): 1.958 M scans/s at 4608 vs 1.918 M at 3840 with the round-6 match;
    # the round-5 match (5 per CU) read 1.892 M at 4608 and 1.906 M at 3840
    # (round 4, same lease: 1.58 M scans/s at 2560 streams, 1.64 M at 3840 -- the update's tail is a smaller
    # share of a longer launch; 1.48 M at 2048: profiles/r04/ab_r04d*.md, ab_r04h_3840.md, r04h_summary.md)
    "northstar": dict(map_size=2048, levels=3, streams=4608),
    # BASELINE configs[1]: single-res 1024^2.  4608 streams (10.5 MB each) = three whole rounds of the match at 6
    # workgroups per CU, like the north star (round 6, one lease: 3840 -> 2.459 M, 4608 -> 2.486 M scans/s,
    # profiles/r06/ab_r06n_c2_fleet.md; round 5 at 5 per CU: 1024 / 2560 / 3840 / 5120 -> 2.17 / 2.47 / 2.53 / 2.49 M)
    "c2": dict(map_size=1024, levels=1, streams=4608),
    # BASELINE configs[2]: 3-level 4096^2
    "c3": dict(map_size=4096, levels=3, streams=1024),  # 1024 x 220 MB pyramids = 225 GB of HBM
}
KERNELS = ("match", "bin", "update")
# the least a once-per-scan update moves per distinct cell it changes: the 4-B log-odds read, the 4-B log-odds
# written and the 2-B update ordinal written (hector_internal.h ORD_OFF; 12 B with round 4's 4-B updateIndex)
FLOOR_BYTES_PER_CELL = 10
PMC_SUMMARY = os.path.join(REPO, "profiles", "pmc_traffic.json")  # written by tools/summarize_profile.py


def kernel_source_id() -> str:
    """16 hex digits of sha256 over the Hector kernel sources: a PMC summary is attached to a bench line
    only when it was taken with the same kernels (tools/summarize_profile.py records it)."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(PKG, "csrc")
    for name in ("hector_kernels.hip", "hector_capi.hip", "hector_internal.h", "detmath.h"):
        try:
            with open(os.path.join(csrc, name), "rb") as f:
                h.update(f.read())
        except OSError:
            return ""
    return h.hexdigest()[:16]


def issue_split() -> str:
    """How a step is issued (part of the PMC workload key: launches per step and streams per launch differ)."""
    return (f"pipeline={os.environ.get('SLAM2D_PIPELINE', '0') or '0'},parts={os.environ.get('SLAM2D_PARTS', '1') or '1'},"
            f"update={os.environ.get('SLAM2D_UPDATE', 'single') or 'single'}")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(ctr: dict, levels: int) -> dict:
    """B_match = Σ_l (1+maxIter_l) N_l 24 B (8 B point + 4 corners x 4 B);
    B_update = ΣL 16 B (8 B LogOddsCell read + 8 B write per traversed cell, ΣL = Σ (abs_da+1))."""
    b_match = ctr["gn_points"] * 24
    b_update = ctr["cells"] * 16
    # hs_bin_kernel: reads every level's points (8 B) and writes the packed end cell (4 B) per ray
    b_bin = ctr["rays"] * 12
    return {"match": b_match, "bin": b_bin, "update": b_update, "total": b_match + b_update,
            "read_only": b_match + ctr["cells"] * 8}


def kernel_symbol(dom: str, ktimes: dict) -> str:
    if dom == "update":
        return "hs_tile_kernel" if ktimes["bin"][1] > 0 else "hs_update_kernel"
    return f"hs_{dom}_kernel"


def pmc_traffic(kernel: str, workload: dict, live_avg_ns: float | None = None):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of this exact
    workload (tools/profile_gpu.sh + tools/summarize_profile.py): FETCH_SIZE x 2 (gfx950 tallies
    128-B read requests at 64 B, MI355X_MICROARCH.md) + WRITE_SIZE, both KB -> bytes.
    workload: config, streams, semantics and reduction order must all match the summary's; a summary
    whose average launch time is more than 25 % away from this run's (another build of the kernel) is
    refused too.  Returns (entry or None, reason)."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_traffic.json"
    # a template kernel is summarised under its instance name (hs_update_kernel<5>); the latest
    # summary of this workload (entries are appended in summary order) wins
    found = None
    for e in d.get("entries", []):
        k = e.get("kernel", "")
        if not (k == kernel or k.startswith(kernel + "<")):
            continue
        if all(e.get(key) == val for key, val in workload.items()):
            found = e
    if found is None:
        return None, f"no PMC summary for {kernel} on this workload {workload}"
    if live_avg_ns and abs(found["avg_ns"] - live_avg_ns) > 0.25 * live_avg_ns:
        return None, (f"PMC summary {found['source']} timed {found['avg_ns'] / 1e3:.1f} us per launch, this run "
                      f"{live_avg_ns / 1e3:.1f} us: another build, not attached")
    return found, found["source"]


def write_calibration():
    """The committed WRITE_SIZE / FETCH_SIZE calibration on the update's store and load shapes
    (tools/probes/write_calib.hip -> profiles/r06/write_calib.json; MI355X_MICROARCH.md's HBM section leaves the
    counters uncalibrated for other widths than 16-B stores): per shape the counted bytes over the 32-B sectors
    written (stores) or over the bytes loaded (2 x FETCH_SIZE).  None when the file is absent."""
    path = os.path.join(REPO, "profiles", "r06", "write_calib.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    ratios = {}
    for r in d.get("shapes", []):
        k = r["kernel"].replace("cal_", "")
        v = r.get("fetch_x2_over_bytes") if k.startswith("ld") else r.get("write_over_sectors32")
        if v is not None:
            ratios[k] = round(v, 4)
    return {"source": "profiles/r06/write_calib.md",
            "meaning": "stores: WRITE_SIZE / (32-B sectors written x 32 B); loads: 2 x FETCH_SIZE / bytes loaded",
            "ratios": ratios}


def aggregate_over_ranks(elapsed: float, units: float, device):
    """Whole-job timing: the slowest rank's time (MAX) and the units all ranks processed (SUM).
    Works on any backend (RCCL on the GPU box, gloo in the CPU tests)."""
    import torch
    import torch.distributed as dist

    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    un = torch.tensor([units], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(un, op=dist.ReduceOp.SUM)
    return float(el.item()), float(un.item())


def launch_ms_max_over_ranks(ktimes: dict, device) -> dict:
    """Average launch time (ms) of every kernel, MAX over ranks (every rank calls this: a collective)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([ktimes[k][0] / max(ktimes[k][1], 1) for k in KERNELS], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return dict(zip(KERNELS, t.tolist()))


def copy_bandwidth(dev, nbytes=2 << 30, reps=5):
    """Attainable device-to-device copy bandwidth (read + write bytes / time), torch copy_."""
    import torch

    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    b.copy_(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        b.copy_(a)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del a, b
    torch.cuda.empty_cache()
    return 2.0 * nbytes * reps / dt / 1e9


def cpu_baseline(cfg, seconds=10.0, seconds_o0=4.0, thresholds=(-1.0, -1.0)):
    """Time the CPU oracle (C restatement at -O3, reference sequential order, 1 core, exactly one
    stream as the reference node runs) on a bounded sample of the same workload: one stream,
    consecutive scans, forced map update each scan.  The -O0 build (the reference ships Debug,
    lesson4/CMakeLists.txt:6) is timed beside it on the same scans."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from slam2d import synth

    n_scans = 600
    S = synth.make_streams(1, n_scans, seed=999)

    def run(variant, budget):
        h = O.HectorOracle(0.05, cfg["map_size"], (0.5, 0.5), cfg["levels"], reduce_threads=0, lib_variant=variant)
        h.set_update_factors(0.4, 0.9)
        h.set_thresholds(*thresholds)
        done = 0
        t0 = time.perf_counter()
        while done < n_scans and time.perf_counter() - t0 < budget:
            h.process(S.points[0, done, : S.counts[0, done]])
            done += 1
        dt = time.perf_counter() - t0
        h.close()
        return done, done / dt

    done, v = run("", seconds)
    done0, v0 = run("O0", seconds_o0)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"value": v, "unit": "scans/s", "cores": 1, "kind": "port",
            "sample": f"1 stream x {done} consecutive synthetic 1081-beam scans, {cfg['map_size']}^2 x "
                      f"{cfg['levels']} levels, {'forced map update' if thresholds[0] < 0 else 'thresholds 0.4 m / 0.9 rad'}, "
                      "oracle/hector_oracle.c -O3 single thread",
            "value_O0": v0, "sample_O0": f"same stream, first {done0} scans, -O0 build", "cpu_model": cpu_model}


def hector_cpu_block(args, cfg, thr, seconds=10.0, seconds_o0=4.0, seconds_all=6.0):
    """The line's cpu_baseline at EVERY GPU count (north_star: the reference CPU path timed "in the same run"):
    rank 0 alone runs it, after the timed region, on 1 core and then on --cpu-cores processes."""
    if args.no_cpu_baseline:
        return None
    cpu = cpu_baseline(cfg, seconds=seconds, seconds_o0=seconds_o0, thresholds=thr)
    if args.cpu_cores > 1:
        cpu["all_cores"] = cpu_baseline_all_cores(cfg, args.cpu_cores, seconds=seconds_all, thresholds=thr)
    return cpu


def _cpu_stream_worker(args):
    """One CPU process = one stream, as the reference node (one spin thread): scans/s of the oracle."""
    map_size, levels, seed, n_scans, budget, thresholds = args
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from slam2d import synth

    S = synth.make_streams(1, n_scans, seed=seed)
    h = O.HectorOracle(0.05, map_size, (0.5, 0.5), levels, reduce_threads=0)
    h.set_update_factors(0.4, 0.9)
    h.set_thresholds(*thresholds)
    done = 0
    t0 = time.perf_counter()
    while done < n_scans and time.perf_counter() - t0 < budget:
        h.process(S.points[0, done, : S.counts[0, done]])
        done += 1
    dt = time.perf_counter() - t0
    h.close()
    return done, dt


def cpu_baseline_all_cores(cfg, procs, seconds=6.0, thresholds=(-1.0, -1.0)):
    """`procs` streams on `procs` cores, one process per core, no sharing; aggregate scans/s."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_stream_worker, [(cfg["map_size"], cfg["levels"], 999 + i, 400, seconds, thresholds)
                                            for i in range(procs)])
    return {"value": sum(d / t for d, t in res), "unit": "scans/s", "cores": procs,
            "sample": f"{procs} processes x 1 stream each, <= {seconds:.0f} s of consecutive scans per process, "
                      "oracle -O3"}


def pose_check(cfg, S, gpu_poses, streams, thresholds=(-1.0, -1.0), order=0):
    """Pose error of the logged GPU streams (device pose log slot i = stream streams[i], every step incl.
    warmup) vs the CPU oracle in the reference's sequential summation order on the same scans -- the
    metric's 'pose RMSE vs ref' -- plus the absolute error against the synthetic ground truth.
    order: the kernel's Hessian summation order (0 = the reference's, the default: the poses must then
    equal the oracle's bit for bit; 256 = the opt-in tree, also compared with the oracle in that order)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    n_scans = gpu_poses.shape[0]
    e, egt, etree = [], [], []
    for i, s in enumerate(streams):
        r = O.HectorOracle(0.05, cfg["map_size"], (0.5, 0.5), cfg["levels"], reduce_threads=0)
        rt = O.HectorOracle(0.05, cfg["map_size"], (0.5, 0.5), cfg["levels"], reduce_threads=order) if order else None
        for h in (r, rt):
            if h is not None:
                h.set_update_factors(0.4, 0.9)
                h.set_thresholds(*thresholds)
        for k in range(n_scans):
            pts = S.points[s, k, : S.counts[s, k]]
            rp, _, _ = r.process(pts)
            e.append(gpu_poses[k, i].astype(np.float64) - rp.astype(np.float64))
            if rt is not None:
                tp, _, _ = rt.process(pts)
                etree.append(gpu_poses[k, i].astype(np.float64) - tp.astype(np.float64))
            egt.append(gpu_poses[k, i].astype(np.float64) - S.gt[s, k])
        r.close()
        if rt is not None:
            rt.close()
    e, egt = np.asarray(e), np.asarray(egt)
    etree = np.asarray(etree) if etree else e
    egt[:, 2] = np.arctan2(np.sin(egt[:, 2]), np.cos(egt[:, 2]))
    # per logged pose: inside the north-star tolerance?  (with the reference order every pose is expected
    # to be EXACT; the tree order reassociates the float sums, and a pose that moves an end cell across a
    # cell boundary changes the map, so later matches can drift apart from there)
    ok = (np.abs(e[:, 0]) <= 1e-4) & (np.abs(e[:, 1]) <= 1e-4) & (np.abs(e[:, 2]) <= 1e-4)
    bad = np.flatnonzero(~ok)
    first = None
    if bad.size:
        i0 = int(bad[0])
        first = {"stream": int(streams[i0 // n_scans]), "scan": int(i0 % n_scans)}
    return {"streams": len(streams), "stream_ids": (f"every 64th of {S.points.shape[0]} and the last"
                                                    if len(streams) > 2 else list(streams)),
            "scans_per_stream": n_scans,
            "rmse_xy_m": float(np.sqrt(np.mean(e[:, 0] ** 2 + e[:, 1] ** 2))),
            "rmse_theta_rad": float(np.sqrt(np.mean(e[:, 2] ** 2))),
            "max_abs_xy_m": float(np.abs(e[:, :2]).max()), "max_abs_theta_rad": float(np.abs(e[:, 2]).max()),
            "tolerance": "1e-4 m / 1e-4 rad (north_star)",
            "within_tolerance_frac": float(ok.mean()), "first_outside_tolerance": first,
            "kernel_summation_order": "reference sequential (OccGridMapUtil.h:94-126)" if not order else f"tree {order}",
            "exact_frac_vs_reference_order": float((np.abs(e).max(axis=1) == 0.0).mean()),
            "vs_oracle_in_kernel_order_max_abs": float(np.abs(etree).max()),
            "vs_oracle_in_kernel_order_exact_frac": float((np.abs(etree).max(axis=1) == 0.0).mean()),
            "vs_ground_truth_rmse_xy_m": float(np.sqrt(np.mean(egt[:, 0] ** 2 + egt[:, 1] ** 2))),
            "vs_ground_truth_rmse_theta_rad": float(np.sqrt(np.mean(egt[:, 2] ** 2)))}


def north_star_targets(value, cpu, roof, pose):
    """BASELINE.json north_star's targets, each with its measured value and pass/fail: >= 100x the
    reference CPU path on 1 GPU (against one core, and against all the box's cores used here), >= 40 % of
    the HBM roofline, pose error <= 1e-4 m / rad.
    The roofline rows are counted bytes only: the dominant kernel's counted HBM traffic (rocprofv3 FETCH_SIZE x 2
    + WRITE_SIZE) and its distinct-cell floor (10 B per distinct cell), each over its launch time.  SURVEY 8d's
    touch model is not a traffic figure (its rate passes the HBM peak, see roofline.survey_8d_note), so it is
    not a target row.  The north star's "HBM-READ roofline" cannot be met by this workload: the update writes
    every cell it reads, so counted reads are at most ~39 % of its counted traffic and a read fraction >= 0.40
    would need more than the HBM peak; read_roofline_counted is reported with that bound beside it."""
    def row(v, target, op, **kw):
        return {"value": None if v is None else round(v, 5), "target": target, "op": op,
                "pass": None if v is None else bool(v >= target if op == ">=" else v <= target), **kw}
    allc = (cpu or {}).get("all_cores")
    roof = roof or {}
    return {"x_cpu_1core": row(value / cpu["value"] if cpu else None, 100.0, ">=", cores=1,
                               basis=(cpu or {}).get("kind")),
            "x_cpu_all_cores": row(value / allc["value"] if allc else None, 100.0, ">=",
                                   cores=allc["cores"] if allc else None, basis="port" if allc else None),
            "hbm_roofline_counted": row(roof.get("frac") if roof.get("traffic") else None, 0.40, ">=",
                                        basis="dominant kernel: counted HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) per "
                                              "launch / avg launch time / 8 TB/s"),
            "hbm_roofline_distinct_cell_floor": row(roof.get("min_traffic_frac"), 0.40, ">=",
                                                    basis="update: 10 B per distinct cell / avg launch time / 8 TB/s"),
            "read_roofline_counted": row(roof.get("read_only_frac_counters"), 0.40, ">=",
                                         basis="rocprofv3 FETCH_SIZE x 2 of the step's kernels / step wall time",
                                         bound=roof.get("read_share_of_counted"),
                                         note="cannot pass: counted reads are `bound` of the step's counted traffic, "
                                              "so even at the HBM peak the read fraction stays below it"),
            "pose_error_m": row(pose["max_abs_xy_m"], 1e-4, "<=", basis="max |GPU - oracle (reference order)|"),
            "pose_error_rad": row(pose["max_abs_theta_rad"], 1e-4, "<=", basis="max |GPU - oracle (reference order)|")}


GM_METRIC = "particle-scans/sec (1081-beam) GMapping ComputeMap, particles sharded over GPUs"


def gmapping_cpu_baseline(seconds=10.0):
    """The REFERENCE's own CPU path: lesson4's GMapping grid headers (G/grid/map.h, harray2d.h,
    gridlinetraversal.h) compiled unmodified into oracle/_ref/libgmapping_ref.so, driven by the
    restated ComputeMap glue (gmapping.cc:171-242), one particle-scan per call, 1 core -- timed without
    any read-out of the map.  The C restatement (oracle/gmapping_oracle.c) is timed beside it."""
    import ctypes as C

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    from slam2d import synth

    ang = synth.beam_angles().astype(np.float64)
    gt = synth.trajectory(8, 0.0)
    ranges = np.ascontiguousarray(synth.cast_ranges(gt[:1], synth.world_segments())[0].astype(np.float32))
    ac, as_ = np.ascontiguousarray(np.cos(ang)), np.ascontiguousarray(np.sin(ang))
    p = O.GM_DEFAULTS

    def timed(call, budget):
        rng = np.random.default_rng(1)
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget and done < 2000:
            x, y, th = gt[0] + rng.normal(0, [0.05, 0.05, 0.02])
            call(x, y, np.cos(th), np.sin(th))
            done += 1
        return done, time.perf_counter() - t0

    out = {}
    if os.path.exists(os.path.join(REPO, "oracle", "_ref", "libgmapping_ref.so")):
        R = O.gmapping_ref_lib()
        nh = C.c_int()
        fp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731

        def ref(x, y, c, s):
            R.gmr_compute_map(x, y, c, s, fp(ranges), ranges.shape[0], fp(ac), fp(as_), p["max_range"],
                              p["max_urange"], p["xmin"], p["ymin"], p["xmax"], p["ymax"], p["delta"], None, None,
                              None, C.byref(nh))
        done, dt = timed(ref, seconds)
        out = {"value": done / dt, "unit": "particle-scans/s", "cores": 1, "kind": "reference",
               "sample": f"{done} ComputeMap calls (1081 beams, fresh 1600^2 ScanMatcherMap each) through the "
                         "reference's own grid headers (oracle/_ref/libgmapping_ref.so, -O3, single thread)"}
    done, dt = timed(lambda x, y, c, s: O.gm_compute(ranges, ac, as_, (x, y, c, s)), seconds / 2)
    port = {"value": done / dt, "unit": "particle-scans/s", "cores": 1, "kind": "port",
            "sample": f"{done} ComputeMap calls, oracle/gmapping_oracle.c -O3 single thread (dense read-out incl.)"}
    if not out:
        return port
    out["port"] = port
    return out


def run_gmapping(args, world, rank, dev):
    """Config 4: every step, each rank runs GMapping::ComputeMap of the step's scan for its shard of
    the particles (poses = ground truth + N(0, [5 cm, 5 cm, 0.02 rad]), seed 777), scores them against
    their previous maps, and normalises the weights of ALL particles with one all-reduce (RCCL)."""
    import torch
    import torch.distributed as dist

    from slam2d import synth
    from slam2d.gmapping import GMappingFleet, RcclComm, normalize_weights

    P_total = args.particles
    P = P_total // world + (1 if rank < P_total % world else 0)
    K, W = args.steps, args.warmup
    T = K + W
    ang = synth.beam_angles().astype(np.float64)
    gt = synth.trajectory(T, 0.0)
    ranges = synth.cast_ranges(gt, synth.world_segments()).astype(np.float32)
    rng = np.random.default_rng(777 + rank)
    noise = rng.normal(0, [0.05, 0.05, 0.02], size=(P, 3))
    d_poses = torch.from_numpy(np.stack([GMappingFleet.poses4(gt[t] + noise) for t in range(T)])).to(dev)
    d_ranges = torch.from_numpy(ranges).to(dev)
    d_scores = torch.zeros(P, dtype=torch.int32, device=dev)
    fleet = GMappingFleet(P)
    fleet.set_beams(ang)
    hs = torch.cuda.current_stream(dev).cuda_stream
    nb = ranges.shape[1]
    c_weights = args.weights == "capi"
    comm = None
    if c_weights and world > 1:
        def bcast(buf):  # the RCCL unique id from rank 0, over the job's process group
            t = torch.from_numpy(buf).to(dev)
            dist.broadcast(t, 0)
            return t.cpu().numpy()
        comm = RcclComm(world, rank, bcast)
    d_w = torch.zeros(P, dtype=torch.float64, device=dev)
    d_sums = torch.zeros(2, dtype=torch.float64, device=dev)

    def step(t):
        fleet.compute_device(d_poses[t].data_ptr(), d_ranges[t].data_ptr(), nb, d_scores.data_ptr(), hip_stream=hs)
        if c_weights:  # gm_normalize_weights_device: ONE RCCL all-reduce of 2 doubles inside the C-ABI
            fleet.normalize_weights_device(comm, d_scores.data_ptr(), P, d_w.data_ptr(), d_sums.data_ptr(), hip_stream=hs)
            return d_w, None
        return normalize_weights(d_scores)

    for t in range(W):
        step(t)
    torch.cuda.synchronize()
    fleet.kernel_times(reset=True)
    fleet.set_timing(not args.no_timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    neff = 0.0
    for t in range(W, T):
        _, neff = step(t)
    torch.cuda.synchronize()
    if neff is None:
        sums = d_sums.cpu().numpy()
        neff = float(sums[0] * sums[0] / sums[1])
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    fleet.set_timing(False)
    kms, kn = fleet.kernel_times(reset=True)
    s, h, f = fleet.scores()
    t_max, total = aggregate_over_ranks(elapsed, float(P * K), dev)
    value = total / t_max
    if rank == 0:
        roof = None
        if kn:
            # per particle-scan Σ(L_b - 1) x 8 B (visits RMW) + hits x 32 B (16-B cell RMW)
            alg = float(f.sum()) * 8 + float(h.sum()) * 32   # last step of this rank's particles
            avg_s = kms / 1e3 / kn
            roof = {"bound": "hbm", "kernel": "gm_compute_kernel", "achieved": round(alg / avg_s / 1e9, 2),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / avg_s / 1e9 / HBM_PEAK_GBS, 5),
                    "traffic": None, "avg_launch_ms": round(kms / kn, 5), "alg_bytes_per_launch": int(alg),
                    "particles_per_launch": P, "free_updates_per_particle": round(float(f.mean()), 1)}
            # counted HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) of the committed rocprofv3 summary of this workload
            tr, src = pmc_traffic("gm_compute_kernel", {"config": "gmapping", "streams": P}, live_avg_ns=avg_s * 1e9)
            roof["traffic_source"] = src
            if tr:
                tb = tr["traffic_bytes_per_launch"]
                roof.update({"traffic": tb, "traffic_over_alg": round(tb / alg, 3),
                             "counted_gbs": round(tb / avg_s / 1e9, 1),
                             "counted_frac": round(tb / avg_s / 1e9 / HBM_PEAK_GBS, 5)})
        cpu = None
        if not args.no_cpu_baseline:  # every GPU count, rank 0 only, after the timed region
            cpu = gmapping_cpu_baseline()
        out = {"metric": GM_METRIC, "value": round(value, 1), "unit": "particle-scans/s", "n_gpus": world, "steps": K,
               "warmup": W, "ms_per_step": round(t_max / K * 1e3, 4), "higher_is_better": True, "scaling": "strong",
               "vs_baseline": None, "dtype": "int32+f64", "data": "synthetic",
               "config": {"workload": f"make_gmapping_map ComputeMap, 1600x1600 @0.05 m fresh map per scan, "
                                      f"{P_total} particles x 1081 beams, weights all-reduced every step",
                          "weights": ("gm_normalize_weights_device (C-ABI, RCCL all-reduce)" if c_weights
                                      else "torch.distributed all_reduce"),
                          "config": "gmapping", "particles": P_total, "particles_per_gpu": P,
                          "parallelism": f"particles sharded x{world}"},
               "roofline": roof, "cpu_baseline": cpu, "neff": neff}
        if cpu:
            out["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    fleet.close()
    if world > 1:
        dist.destroy_process_group()

PL_METRIC = "scan-pairs/sec (1081-beam) PL-ICP sm_icp (lesson3 parameters)"


def plicp_pairs(num, seed, noise=0.01):
    """Consecutive synthetic scans as LDP readings (LaserScanToLDP: -1 outside (0.1, 29.9) m)."""
    from slam2d import synth
    from slam2d.plicp import laser_scan_to_readings

    rng = np.random.default_rng(seed)
    phase = rng.uniform(0, 6.28)
    gt = synth.trajectory(num + 1, phase)
    R = synth.cast_ranges(gt, synth.world_segments()) + rng.normal(0, noise, (num + 1, synth.N_BEAMS))
    R = laser_scan_to_readings(R, 0.1, 29.9)
    ang = synth.beam_angles().astype(np.float64)
    return R, float(ang[0]), float(ang[1] - ang[0])


def plicp_cpu_baseline(seconds=10.0):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    R, amin, inc = plicp_pairs(400, 4242)
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < 400:
        O.plicp(R[done], R[done + 1], amin, inc)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "scan-pairs/s", "cores": 1, "kind": "port",
            "sample": f"{done} consecutive synthetic 1081-beam scan pairs, oracle/plicp_oracle.c -O3 single thread "
                      "(exact polar-interval search; CSM's use_corr_tricks search is not available here)"}


def run_plicp(args, world, rank, dev):
    """lesson3 front-end: every step runs sm_icp for B independent scan pairs per GPU (B odometry
    streams), inputs resident in HBM; replicas across GPUs (no exchange)."""
    import torch
    import torch.distributed as dist

    from slam2d.plicp import PLICP

    B, K, W = args.pairs, args.steps, args.warmup
    R, amin, inc = plicp_pairs(B + K + W, 777 + rank)
    d_R = torch.from_numpy(R).to(dev)
    d_guess = torch.zeros((B, 3), dtype=torch.float64, device=dev)
    d_out = torch.zeros((B, 48), dtype=torch.uint8, device=dev)
    pl = PLICP(B, R.shape[1])
    hs = torch.cuda.current_stream(dev).cuda_stream
    nb = R.shape[1]
    row = nb * 8

    def step(t):  # pairs (t + b, t + b + 1), b < B: each pair a different stream position
        pl.icp_batch_device(B, nb, amin, inc, d_R.data_ptr() + t * row, d_R.data_ptr() + (t + 1) * row,
                            d_guess.data_ptr(), d_out.data_ptr(), hip_stream=hs)

    for t in range(W):
        step(t)
    torch.cuda.synchronize()
    pl.kernel_times(reset=True)
    pl.set_timing(not args.no_timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(W, W + K):
        step(t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    pl.set_timing(False)
    kms, kn = pl.kernel_times(reset=True)
    t_max, total = aggregate_over_ranks(elapsed, float(B * K), dev)
    if rank == 0:
        cpu = None if args.no_cpu_baseline else plicp_cpu_baseline()
        out = {"metric": PL_METRIC, "value": round(total / t_max, 1), "unit": "scan-pairs/s", "n_gpus": world,
               "steps": K, "warmup": W, "ms_per_step": round(t_max / K * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": {"workload": f"lesson3 plicp_odometry sm_icp, {B} independent 1081-beam scan pairs per GPU, "
                                      "point-to-line, max 10 iterations", "config": "plicp", "pairs_per_gpu": B,
                          "parallelism": f"replicas x{world}"},
               "roofline": ({"bound": "latency", "kernel": "pl_icp_kernel", "avg_launch_ms": round(kms / kn, 5),
                             "note": "compute/latency bound (no HBM roofline: 17 KB of input per pair)"}
                            if kn else None),
               "cpu_baseline": cpu}
        if cpu:
            out["speedup_vs_cpu_1core"] = round(out["value"] / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    pl.close()
    if world > 1:
        dist.destroy_process_group()

KT_METRIC = {"karto": "matches/sec Karto ScanMatcher::MatchScan (coarse 16x16x21 + fine 3x3x11, 10 running scans)",
             "karto_loop": "loop-closure matches/sec Karto ScanMatcher::MatchScan (coarse 101x101x21, 10-scan chain)"}


def karto_setup(cfg, M, seed):
    """Pool + batch description for one GPU.  karto: M sequential matches, each against the 10 scans
    before it (running scans, Mapper.cpp:2040); karto_loop: M loop-closure candidates, each against a
    10-scan chain from the first lap (TryCloseLoop's coarse call, Mapper.cpp:991)."""
    import math

    from slam2d import karto, synth

    lz = karto.laser(synth.N_BEAMS, float(synth.ANGLE_MIN), float(synth.ANGLE_INC), 0.1, 12.0)
    if cfg == "karto":
        K = 10
        R, T, Q = synth.karto_sequential(M, K, seed=seed)
        ranges = np.concatenate([R, R[K:]])
        poses = np.concatenate([T, Q[K:]])
        query = np.arange(M + K, 2 * M + K, dtype=np.int32)
        beg = (np.arange(M + 1) * K).astype(np.int32)
        idx = (np.arange(M)[:, None] + np.arange(K)[None, :]).reshape(-1).astype(np.int32)
        p = karto.default_params()
        penalize, refine = True, True
    else:
        K = 10
        QR, qp, qt, CR, CP = synth.karto_loop(M, K, seed=seed)
        ranges = np.concatenate([QR, CR.reshape(-1, synth.N_BEAMS)])
        poses = np.concatenate([qp, CP.reshape(-1, 3)])
        query = np.arange(M, dtype=np.int32)
        beg = (np.arange(M + 1) * K).astype(np.int32)
        idx = (M + np.arange(M * K)).astype(np.int32)
        p = karto.default_params(loop=True)
        p.search_size = 10.0  # 101 x 101 x 21 coarse window at 0.05 m
        penalize, refine = False, False
    return lz, p, ranges, poses, query, beg, idx, K, penalize, refine


def karto_cpu_baseline(cfg, seconds=10.0):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O

    lz, p, ranges, poses, query, beg, idx, K, pen, ref = karto_setup(cfg, 32, 4242)
    ol = O.KtLaser(lz.minimum_angle, lz.angular_resolution, lz.minimum_range, lz.range_threshold, lz.n_readings, 0)
    op = O.KtParams(*[getattr(p, f) for f, _ in p._fields_])
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < len(query):
        b = idx[beg[done]:beg[done + 1]]
        O.karto_match(ol, op, ranges[query[done]], poses[query[done]], ranges[b], poses[b], pen, ref)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "matches/s", "cores": 1, "kind": "port",
            "sample": f"{done} synthetic {cfg} matches (1081 beams, {K} base scans), oracle/karto_oracle.c -O3 "
                      "single thread (sequential restatement of open_karto's ScanMatcher; the library itself needs "
                      "boost and is not built here)"}


def run_karto(args, world, rank, dev):
    """Karto correlative matcher (config 5): every step prepares the pool's scans (point readings) and
    runs M independent MatchScan calls per GPU, inputs resident in HBM; replicas across GPUs."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    from slam2d import karto

    cfg = args.config
    # matches per GPU per step (end-of-round-2 sweep: sequential 512 / 1024 / 2048 -> 321 k / 375 k / 387 k
    # matches/s, loop window 32 / 64 / 128 -> 22.2 k / 25.0 k / 25.6 k: small batches leave the launches' tails)
    M = args.matches or (2048 if cfg == "karto" else 128)
    K, W = args.steps, args.warmup
    shard = args.karto_shard
    # replicas: every rank its own matches; sharded: every rank the SAME matches, window split by angle
    lz, p, ranges, poses, query, beg, idx, NB, pen, ref = karto_setup(cfg, M, 777 + (0 if shard else rank))
    S = ranges.shape[0]
    sm = karto.ScanMatcher(lz, p, max_matches=M, max_scans=S, max_base=NB)
    d_r = torch.from_numpy(ranges).to(dev)
    d_p = torch.from_numpy(poses).to(dev)
    d_q, d_b, d_i = (torch.from_numpy(a).to(dev) for a in (query, beg, idx))
    d_res = torch.zeros(M * C.sizeof(karto.KtResult), dtype=torch.uint8, device=dev)
    hs = torch.cuda.current_stream(dev).cuda_stream

    def step():
        sm.set_scans_device(0, S, d_r.data_ptr(), d_p.data_ptr(), hip_stream=hs)
        if shard:  # one RCCL all-reduce (MAX) of the window's exchange words per step
            sm.match_sharded(M, d_q.data_ptr(), d_b.data_ptr(), d_i.data_ptr(), d_res.data_ptr(), pen, ref)
        else:
            sm.match_batch_device(M, d_q.data_ptr(), d_b.data_ptr(), d_i.data_ptr(), d_res.data_ptr(), pen, ref,
                                  hip_stream=hs)

    for _ in range(W):
        step()
    torch.cuda.synchronize()
    sm.kernel_times(reset=True)
    sm.set_timing(not args.no_timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sm.set_timing(False)
    kt = sm.kernel_times(reset=True)
    res = karto.results_from_bytes(d_res.cpu().numpy())
    t_max, total = aggregate_over_ranks(elapsed, float(M * K), dev)
    if shard:
        total = float(M * K)  # the same matches on every rank: the job's matches, not the ranks' sum
    if rank == 0:
        cpu = None if args.no_cpu_baseline else karto_cpu_baseline(cfg)
        info = sm.info
        coarse_ms, coarse_n = kt.get("kt_coarse_kernel", (0.0, 0))
        nA = 21
        npos = ((info["side"] - 1) // 2 + 1) ** 2
        roof = None
        if coarse_n and not args.no_timing:
            # algorithmic bytes of one coarse launch: every (pose, point) lookup reads one grid byte,
            # plus the 16-byte local point and 1-byte flag each (angle, tile) workgroup reads per point
            tiles = -(-int(math.sqrt(npos)) // 16) ** 2
            pts = float(np.isfinite(ranges[query]).sum(axis=1).mean())
            nA_own = sum(1 for a in range(nA) if karto.shard_owns_angle(a, rank, world)) if shard else nA
            per_launch = M * (npos * nA_own * pts + nA_own * tiles * pts * 17.0)
            avg_s = coarse_ms / coarse_n * 1e-3
            ach = per_launch / avg_s / 1e9
            # the correlation grids are cache resident, so the gather rate is priced against the measured gather
            # rate of the cache level that holds them (MI355X_MICROARCH.md, 'Indexed rows: gather into LDS':
            # rows shared by every workgroup from the XCD's L2 16.8-18.8 TB/s, a 38 MB table from the Infinity
            # Cache 8.6 TB/s), not against the HBM peak; the lower bound of the range is the peak used
            # the level: every grid of the launch in one XCD's L2 (4 MiB); else each match's grid (read by that match's
            # angle x tile workgroups, which run together) inside the 256 MiB Infinity Cache; else HBM
            grid_bytes = float(M) * float(info["grid_size"]) ** 2
            match_grid = float(info["grid_size"]) ** 2
            level = "l2" if grid_bytes <= 4.0 * 2 ** 20 else ("infinity_cache" if match_grid <= 256.0 * 2 ** 20 else "hbm")
            peak = {"l2": 16800.0, "infinity_cache": 8600.0, "hbm": HBM_PEAK_GBS}[level]
            roof = {"bound": level, "kernel": "kt_coarse_kernel", "achieved": round(ach, 1),
                    "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 4), "traffic": None,
                    "avg_launch_ms": round(coarse_ms / coarse_n, 5), "grid_bytes_per_launch": int(grid_bytes),
                    "grid_bytes_per_match": int(match_grid),
                    "frac_of_hbm_peak": round(ach / HBM_PEAK_GBS, 4),
                    "note": "achieved = lookup bytes (1 B per pose x point) / launch time: a cache gather rate, not "
                            "DRAM traffic; peak = the guide's measured gather rate of the level holding the grids"}
        out = {"metric": KT_METRIC[cfg], "value": round(total / t_max, 1), "unit": "matches/s", "n_gpus": world,
               "steps": K, "warmup": W, "ms_per_step": round(t_max / K * 1e3, 4), "higher_is_better": True,
               "scaling": "strong" if shard else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
               "config": {"workload": f"lesson6 karto_slam {cfg}: {M} independent MatchScan calls "
                                      f"{'per job, coarse window split over the GPUs by angle' if shard else 'per GPU'}, "
                                      f"{NB} base scans each, 1081 beams, grid {info['grid_size']}^2",
                          "config": cfg, "matches_per_gpu": M,
                          "parallelism": f"window sharded x{world} (RCCL MAX all-reduce)" if shard else f"replicas x{world}",
                          "kernel_ms": {k: round(v[0], 3) for k, v in kt.items()}},
               "roofline": roof, "cpu_baseline": cpu,
               "ok_results": int((res["status"] == 0).sum())}
        if cpu:
            out["speedup_vs_cpu_1core"] = round(out["value"] / cpu["value"], 1)
        print(json.dumps(out), flush=True)
    sm.close()
    if world > 1:
        dist.destroy_process_group()


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` (N > 1) without an external launcher: start N ranks, one process per GPU, as
    `python -m torch.distributed.run --nproc-per-node N bench.py <same args>` on 127.0.0.1 (a child
    process -- this parent makes no HIP / torch.cuda call and never execs), relay rank 0's JSON line and
    return the launcher's exit code (non-zero when any rank failed)."""
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"[bench] launching {n} ranks: {' '.join(cmd[2:])}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for ln in p.stdout:  # only rank 0 prints to stdout (one JSON line); anything else goes to stderr
        if ln.startswith("{"):
            sys.stdout.write(ln)
            sys.stdout.flush()
        else:
            sys.stderr.write(ln)
    return p.wait()


def launcher_selftest(args):
    """Rank body of the launcher's CPU test (no GPU): gloo all-reduce of every rank's unit count, rank 0
    prints the job's line as the benchmarks do."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    t_max, total = aggregate_over_ranks(time.perf_counter() - t0 + 1e-3, float(args.streams or 1), torch.device("cpu"))
    if rank == 0:
        # the Hector line's CPU block exactly as main() builds it at any world size (short budgets, c2's grid)
        cpu = hector_cpu_block(args, CONFIGS["c2"], (-1.0, -1.0), seconds=0.5, seconds_o0=0.2, seconds_all=0.5)
        print(json.dumps({"metric": "launcher-selftest", "value": total / t_max, "unit": "units/s", "n_gpus": world,
                          "config": {"global_batch": int(total), "ranks": world}, "cpu_baseline": cpu}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=0, help="streams per GPU (0 = config default)")
    ap.add_argument("--config", default="northstar", choices=sorted(CONFIGS) + ["gmapping", "plicp", "karto", "karto_loop"])
    ap.add_argument("--pairs", type=int, default=8192,
                    help="plicp: scan pairs per GPU per step (2048 / 4096 / 8192: 1.49 / 1.61 / 1.69 M pairs/s)")
    ap.add_argument("--matches", type=int, default=0, help="karto: MatchScan calls per GPU per step (0 = default)")
    ap.add_argument("--particles", type=int, default=1024, help="gmapping: particles of the whole job")
    ap.add_argument("--weights", choices=["capi", "torch"], default="capi",
                    help="gmapping: particle-weight exchange through gm_normalize_weights_device (RCCL inside the "
                         "C-ABI) or the Python torch.distributed path")
    ap.add_argument("--karto-shard", action="store_true",
                    help="karto: split every match's coarse window over the GPUs (one RCCL all-reduce per step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--no-copy-probe", action="store_true", help="skip the copy-bandwidth probe")
    ap.add_argument("--order", choices=["reference", "tree"], default="reference",
                    help="hector: Hessian summation order of the matcher (the reference's sequential order, default; "
                         "or the faster 256-thread tree)")
    ap.add_argument("--semantics", choices=["forced", "reference"], default="forced",
                    help="hector: map update every scan (benchmark mode, SURVEY.md 8d) or the node's thresholds "
                         "0.4 m / 0.9 rad (reference semantics, reported separately)")
    ap.add_argument("--cpu-cores", type=int, default=16,
                    help="processes for the all-core CPU baseline (one stream each; the GPU box's CPU share is 16)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="hector ranges input: one hs_step_ranges_batch_device call per step instead of one "
                         "K-step hs_run_ranges_device call")
    ap.add_argument("--input", choices=["ranges", "points"], default="ranges",
                    help="hector: raw LaserScan ranges through the on-device ingest (scanCallback, default) or "
                         "pre-converted DataContainer points")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    # --gpus N: the driver launches N > 1 ranks with torch.distributed.run (WORLD_SIZE set, = N); a bare
    # `bench.py --gpus N` starts them itself (launch_ranks) before anything touches the GPU
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}: refusing a mislabelled run",
              file=sys.stderr, flush=True)
        return 2
    if args.launcher_selftest:
        return launcher_selftest(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one rank per GPU over RCCL (the driver's node).  BENCH_DIST_BACKEND=gloo rehearses the N > 1 path
        # with several ranks on one GPU (RCCL refuses two ranks on one device): timing collectives on gloo
        dev_idx = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev_idx)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from slam2d import synth
    from slam2d.hector import HectorFleet

    if args.config == "gmapping":
        return run_gmapping(args, world, rank, dev)
    if args.config == "plicp":
        return run_plicp(args, world, rank, dev)
    if args.config in ("karto", "karto_loop"):
        return run_karto(args, world, rank, dev)
    cfg = dict(CONFIGS[args.config])
    B = args.streams or cfg["streams"]
    K, W = args.steps, args.warmup
    # the headline pass (K steps) runs without per-kernel events (they add ~15 us of gaps per step on
    # MI355X); the kernel durations for the roofline come from a second, instrumented pass of K more steps
    P = 0 if args.no_timing else K
    T = K + W + P

    # ---- synthetic input, resident in HBM before timing: [step][stream][1081][2] ----
    t0 = time.perf_counter()
    S = synth.make_streams(B, T, seed=12345 + rank * B)
    from_ranges = args.input == "ranges"
    if from_ranges:  # LaserScan ranges [step][stream][1081] float32
        rng_in = np.ascontiguousarray(S.ranges.transpose(1, 0, 2))
        d_rng = torch.from_numpy(rng_in).to(dev)
    else:
        pts = np.ascontiguousarray(S.points.transpose(1, 0, 2, 3))
        cnt = np.ascontiguousarray(S.counts.T.astype(np.int32))
        d_pts = torch.from_numpy(pts).to(dev)
        d_cnt = torch.from_numpy(cnt).to(dev)
    log(f"[bench] rank {rank}: generated {B} streams x {T} scans in {time.perf_counter() - t0:.1f}s")

    fleet = HectorFleet(B, 0.05, cfg["map_size"], (0.5, 0.5), cfg["levels"], max_points=1081)
    fleet.set_update_factors(0.4, 0.9)   # hector_slam.cc:144-145
    ref_sem = args.semantics == "reference"
    thr = (0.4, 0.9) if ref_sem else (-1.0, -1.0)
    fleet.set_thresholds(*thr)           # benchmark mode: update every scan; reference: hector_slam.launch
    if args.order == "tree":
        fleet.set_reduction_order(HectorFleet.ORDER_TREE256)
    order = fleet.reduction_order()
    # the source hash compiled into the loaded library (hs_source_id): the line names the binary it timed, and
    # says whether csrc/ still holds that source (a stale library is marked, not silently attributed)
    from slam2d import _lib
    lib_src, tree_src = _lib.source_id_of_library(), kernel_source_id()
    if lib_src != tree_src:
        log(f"[bench] WARNING: {_lib.LIB_PATH} was built from Hector sources {lib_src}, csrc/ holds {tree_src}")
    workload = {"config": args.config, "streams": B, "semantics": args.semantics, "order": order,
                "kernel_src": lib_src, "issue_split": issue_split()}
    hs = torch.cuda.current_stream(dev).cuda_stream
    # pose log: every 64th stream and the last one (the top of the update lists and of the HBM range)
    log_streams = sorted(set(range(0, B, 64)) | {B - 1})
    slot_of = np.full(B, -1, np.int32)
    slot_of[log_streams] = np.arange(len(log_streams), dtype=np.int32)
    d_slot = torch.from_numpy(slot_of).to(dev)
    d_plog = torch.zeros((T, len(log_streams), 3), dtype=torch.float32, device=dev)
    fleet.set_pose_log_slots(d_plog.data_ptr(), d_slot.data_ptr(), len(log_streams), T)
    if from_ranges:
        # the node's filters with the generator's own beam directions as the unit-vector cache, so the
        # device DataContainers equal synth's points (the pose check below replays those)
        from slam2d.hector import HsLaser
        nb = S.ranges.shape[2]
        ang = synth.beam_angles(nb)
        fleet.set_laser(HsLaser.defaults(nb, float(ang[0]), float(ang[1] - ang[0])),
                        unit_vectors=np.stack([np.cos(ang), np.sin(ang)], 1))

        def step(t):
            fleet.step_ranges_device(d_rng[t].data_ptr(), nb, hip_stream=hs)

        def run(t, k):  # k consecutive steps from step t, pipelined inside the library
            fleet.run_ranges_device(k, d_rng[t].data_ptr(), nb, B * nb, hip_stream=hs)
    else:
        stride = pts.shape[2]
        step_bytes = pts.shape[1] * pts.shape[2] * 8

        def step(t):
            fleet.step_device(d_pts.data_ptr() + t * step_bytes, stride, d_cnt[t].data_ptr(), hip_stream=hs)

    pipelined = from_ranges and not args.no_pipeline
    if pipelined:
        run(0, W)
    else:
        for t in range(W):
            step(t)
    torch.cuda.synchronize()
    fleet.counters(reset=True)
    fleet.kernel_times(reset=True)
    fleet.set_timing(False)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if pipelined:
        run(W, K)
    else:
        for t in range(W, W + K):
            step(t)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctr = fleet.counters(reset=True)

    # instrumented pass: the same K-step workload on the next K scans, HIP events around every kernel
    # on the stream it is launched on (the library's timing events)
    ktimes, ctr_i, elapsed_i = None, None, None
    clk = None
    if P:
        fleet.set_timing(True)
        fleet.set_clock_probe(True)   # effective shader clock of the instrumented pass (s_memtime / s_memrealtime)
        fleet.clock_probe(reset=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if pipelined:
            run(W + K, P)
        else:
            for t in range(W + K, T):
                step(t)
        torch.cuda.synchronize()
        elapsed_i = time.perf_counter() - t1
        fleet.set_timing(False)
        clk = fleet.clock_probe(reset=True)
        fleet.set_clock_probe(False)
        ktimes = fleet.kernel_times(reset=True)
        ctr_i = fleet.counters(reset=True)

    t_max, total_scans = aggregate_over_ranks(elapsed, float(B * K), dev)
    value = total_scans / t_max
    # per-launch kernel times, MAX over ranks (the roofline's launch time is the slowest rank's)
    kmax = launch_ms_max_over_ranks(ktimes, dev) if ktimes else None

    if rank == 0:
        ab = algorithmic_bytes(ctr, cfg["levels"])
        roof = None
        if ktimes and ktimes["update"][1] > 0:
            ab_i = algorithmic_bytes(ctr_i, cfg["levels"])
            dom = max(KERNELS, key=lambda k: ktimes[k][0])
            ms, nlaunch = ktimes[dom]
            ms = kmax[dom] * nlaunch  # the slowest rank's launches (= rank 0's at N = 1)
            avg_s = ms / 1e3 / nlaunch
            ksym = kernel_symbol(dom, ktimes)
            pmc, pmc_why = pmc_traffic(ksym, workload, avg_s * 1e9)
            # distinct-cell floor of the update: every cell the scan changes is read once (4 B log-odds)
            # and written once (4 B log-odds + 2 B update ordinal) -- the least this layout's update moves
            floor = ctr_i["touched"] * FLOOR_BYTES_PER_CELL / nlaunch if dom == "update" else ab_i[dom] / nlaunch
            model_8d = ab_i[dom] / nlaunch
            # achieved / frac: counted HBM bytes (PMC summary of this exact workload) when available, else
            # the distinct-cell floor -- both are bytes the kernel really moves, so frac <= 1.  SURVEY 8d's
            # touch model (16 B per cell touch, re-touches by later beams included, which the kernel merges
            # in LDS) is reported as bytes only.
            moved = pmc["traffic_bytes_per_launch"] if pmc else floor
            achieved = moved / avg_s / 1e9
            mpmc, _ = pmc_traffic("hs_match_kernel", workload, None)
            roof = {"bound": "hbm", "kernel": ksym, "achieved": round(achieved, 2),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                    "traffic": pmc["traffic_bytes_per_launch"] if pmc else None,
                    "achieved_basis": ("PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE) / avg launch time; the "
                                       "counters calibrated on the update's own shapes (traffic_calibration): WRITE_SIZE "
                                       "is the 32-B sectors written, 2 x FETCH_SIZE the bytes of its 16-B loads"
                                       if pmc else "distinct-cell floor (10 B per distinct cell) / avg launch time"),
                    "traffic_calibration": write_calibration(),
                    "traffic_source": (f"{pmc_why} (FETCH_SIZE x2 + WRITE_SIZE)" if pmc else pmc_why),
                    "min_traffic_per_launch": int(floor) if dom == "update" else None,
                    "min_traffic_frac": (round(floor / avg_s / 1e9 / HBM_PEAK_GBS, 5) if dom == "update" else None),
                    "traffic_over_floor": (round(pmc["traffic_bytes_per_launch"] / floor, 3) if pmc and dom == "update"
                                           else None),
                    "survey_8d_bytes_per_launch": int(model_8d),
                    "survey_8d_note": ("SURVEY 8d: 16 B per cell touch of the reference's raycast (8 B LogOddsCell read "
                                       "+ write), re-touches of a cell by later beams included; the kernel merges them "
                                       "in LDS and moves each distinct cell once, so this is work, not traffic")
                    if dom == "update" else None,
                    "avg_launch_ms": round(ms / nlaunch, 5),
                    "avg_launch_ms_basis": "max over ranks" if world > 1 else "rank 0",
                    "timing": "kernel durations from an instrumented pass of K further steps (HIP events "
                              "around each kernel); the headline pass runs without events",
                    "instrumented_ms_per_step": round(elapsed_i / P * 1e3, 4),
                    "kernel_ms_per_step": {k: round(ktimes[k][0] / max(ktimes[k][1], 1), 5) for k in KERNELS},
                    # the north star's "HBM-read roofline": SURVEY 8d's read subset (match gathers + 8 B per cell
                    # touch; a touch model, not traffic) over the step's wall time, and the counted reads of the
                    # step's kernels (PMC) with their share of the step's counted traffic (the bound on that fraction)
                    "survey_8d_read_only_frac": round(ab["read_only"] / t_max / 1e9 / HBM_PEAK_GBS, 5),
                    # counted reads per launch x launches per step (ktimes over the P instrumented steps) x K
                    "read_share_of_counted": (round(2 * (pmc["fetch_kb"] * ktimes["update"][1] + mpmc["fetch_kb"]
                                                         * ktimes["match"][1]) * 1024
                                                    / (pmc["traffic_bytes_per_launch"] * ktimes["update"][1]
                                                       + mpmc["traffic_bytes_per_launch"] * ktimes["match"][1]), 4)
                                              if (pmc and mpmc and dom == "update") else None),
                    "read_only_frac_counters": (round(2 * (pmc["fetch_kb"] * ktimes["update"][1] + mpmc["fetch_kb"]
                                                           * ktimes["match"][1]) / P * 1024 * K
                                                      / t_max / 1e9 / HBM_PEAK_GBS, 5)
                                                if (pmc and mpmc and dom == "update") else None),
                    "alg_bytes_per_scan": int(ab["total"] / max(B * K, 1)),
                    "cells_per_scan": round(ctr["cells"] / max(B * K, 1), 1),
                    "distinct_cells_per_scan": round(ctr["touched"] / max(B * K, 1), 1)}
            if clk:
                # effective shader clock over the instrumented pass (every 16th workgroup's lifetime): kernel
                # times compare across boxes as cycles = ms x clock
                ck = clk["update" if dom == "update" else "match"]
                roof["sclk_mhz"] = ck["sclk_mhz"]
                roof["match_sclk_mhz"] = clk["match"]["sclk_mhz"]
                roof["update_sclk_mhz"] = clk["update"]["sclk_mhz"]
                if ck["sclk_mhz"]:
                    roof["mcycles_per_launch"] = round(ms / nlaunch * 1e-3 * ck["sclk_mhz"], 3)
                roof["clock_probe"] = clk
            for kk, ent in (("update", pmc), ("match", mpmc)):
                # instruction counts per launch from the committed PMC summary of this workload (when taken)
                if ent and ent.get("insts_valu") is not None:
                    roof.setdefault("pmc_insts_per_launch", {})[kk] = {
                        c: ent.get(c) for c in ("insts_valu", "insts_salu", "insts_lds", "wave_cycles", "busy_cycles")}
            if not args.no_copy_probe:
                roof["attainable_copy_GBps"] = round(copy_bandwidth(dev), 1)
        cpu = hector_cpu_block(args, cfg, thr)
        pose = pose_check(cfg, S, d_plog.cpu().numpy(), log_streams, thresholds=thr, order=order)
        out = {"metric": METRIC, "value": round(value, 1), "unit": "scans/s", "n_gpus": world, "steps": K,
               "warmup": W, "ms_per_step": round(t_max / K * 1e3, 4), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
               "config": {"workload": f"hector_slam match+update, {cfg['map_size']}x{cfg['map_size']} @0.05 m x "
                                      f"{cfg['levels']} levels, 1081-beam scans, "
                                      + ("reference map-update thresholds 0.4 m / 0.9 rad" if ref_sem
                                         else "map update every scan"),
                          "config": args.config, "streams_per_gpu": B, "global_batch": B * world,
                          "map_size": cfg["map_size"], "levels": cfg["levels"], "beams": 1081,
                          "input": ("LaserScan ranges (on-device ingest in the timed region)" if from_ranges
                                    else "DataContainer points"),
                          "issue": (("hs_run_ranges_device: K steps in one call"
                                     + (", two fleet halves pipelined (SLAM2D_PIPELINE=1)"
                                        if os.environ.get("SLAM2D_PIPELINE", "0") not in ("", "0") else ""))
                                    if pipelined else "one batch call per step"),
                          "parallelism": f"replicas x{world}", "semantics": args.semantics,
                          "reduction_order": order, "kernel_src": workload["kernel_src"],
                          "kernel_src_of": "hs_source_id() of the loaded library",
                          "kernel_src_matches_tree": lib_src == tree_src,
                          "issue_split": workload["issue_split"],
                          "map_updates_per_scan": round(ctr["updates"] / max(B * K, 1), 4)},
               "roofline": roof, "cpu_baseline": cpu, "pose_vs_ref": pose}
        if cpu:
            out["speedup_vs_cpu_1core"] = round(value / cpu["value"], 1)
        out["targets"] = north_star_targets(value, cpu, roof, pose)
        print(json.dumps(out), flush=True)
    fleet.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
