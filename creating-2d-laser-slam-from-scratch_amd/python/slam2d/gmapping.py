"""GMapping particle-map path over the MI355X C-ABI (include/slam2d/gmapping.h).

Reference: lesson4 `make_gmapping_map` -- GMapping::ComputeMap (lesson4/src/gmapping/gmapping.cc:
171-242) into a fresh ScanMatcherMap per scan, PublishMap (:141-159), CreateCache (:111-124).
`GMappingFleet` evaluates one scan for P candidate poses ("particles") resident on one GPU; the
particles of a multi-GPU job are sharded over ranks and their scores normalised with one RCCL
all-reduce (`normalize_weights`).  Every compute call goes to the HIP library; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import Slam2dError


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _check(L, rc: int, what: str):
    if rc != 0:
        raise Slam2dError(f"{what} failed with code {rc}: {L.gm_last_error().decode(errors='replace')}")


# gmapping.cc ctor defaults / launch parameters: +-40 m map at 0.05 m,
# maxRange 30 - 0.01, maxUrange 25, occ_thresh 0.25
DEFAULTS = dict(xmin=-40.0, ymin=-40.0, xmax=40.0, ymax=40.0, delta=0.05, max_range=30.0 - 0.01, max_urange=25.0)


class GMappingFleet:
    """P particle maps of GMapping::ComputeMap on one GPU."""

    def __init__(self, num_particles: int, max_beams: int = 1081, **params):
        p = dict(DEFAULTS)
        p.update(params)
        self.L = _lib.lib()
        self.P = num_particles
        self.h = C.c_void_p()
        _check(self.L, self.L.gm_create(C.byref(self.h), num_particles, max_beams, p["xmin"], p["ymin"], p["xmax"],
                                        p["ymax"], p["delta"], p["max_range"], p["max_urange"]), "gm_create")
        sx, sy = C.c_int(), C.c_int()
        self.L.gm_get_map_size(self.h, C.byref(sx), C.byref(sy))
        self.size = (sx.value, sy.value)
        self.n_beams = 0

    def close(self):
        if self.h:
            self.L.gm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        _check(self.L, self.L.gm_reset(self.h), "gm_reset")

    def set_beams(self, angles=None, a_cos=None, a_sin=None):
        """GMapping::CreateCache (gmapping.cc:111-124): cos/sin of every beam angle (double)."""
        if angles is not None:
            angles = np.asarray(angles, np.float64)
            a_cos, a_sin = np.cos(angles), np.sin(angles)
        a_cos = np.ascontiguousarray(a_cos, np.float64)
        a_sin = np.ascontiguousarray(a_sin, np.float64)
        _check(self.L, self.L.gm_set_beams(self.h, _fp(a_cos), _fp(a_sin), a_cos.shape[0]), "gm_set_beams")
        self.n_beams = a_cos.shape[0]

    def set_occ_thresh(self, t: float):
        _check(self.L, self.L.gm_set_occ_thresh(self.h, float(t)), "gm_set_occ_thresh")

    @staticmethod
    def poses4(poses_xyt) -> np.ndarray:
        """(x, y, theta) -> (x, y, cos theta, sin theta) as the kernel consumes them."""
        p = np.asarray(poses_xyt, np.float64).reshape(-1, 3)
        return np.ascontiguousarray(np.stack([p[:, 0], p[:, 1], np.cos(p[:, 2]), np.sin(p[:, 2])], axis=1))

    def compute(self, poses4, ranges):
        """ComputeMap for every particle (host arrays, synchronous)."""
        poses4 = np.ascontiguousarray(poses4, np.float64).reshape(self.P, 4)
        ranges = np.ascontiguousarray(ranges, np.float32)
        _check(self.L, self.L.gm_compute_maps(self.h, _fp(poses4), _fp(ranges), ranges.shape[0]), "gm_compute_maps")

    def compute_device(self, d_poses4: int, d_ranges: int, n: int, d_scores: int = 0, begin: int = 0,
                       count: int | None = None, hip_stream: int = 0):
        count = self.P - begin if count is None else count
        _check(self.L, self.L.gm_compute_maps_device(self.h, begin, count, C.c_void_p(d_poses4), C.c_void_p(d_ranges),
                                                     int(n), C.c_void_p(d_scores or None),
                                                     C.c_void_p(hip_stream or None)), "gm_compute_maps_device")

    def normalize_weights_device(self, comm, d_scores: int, count: int, d_weights: int, d_sums: int,
                                 hip_stream: int = 0):
        """gm_normalize_weights_device: [Σ(s+1), Σ(s+1)^2] of this rank's scores all-reduced with RCCL on
        `comm` (an RcclComm or None for a single rank), weights (double[count]) and sums (double[2])."""
        _check(self.L, self.L.gm_normalize_weights_device(self.h, C.c_void_p(comm.handle if comm else None),
                                                          C.c_void_p(d_scores), int(count),
                                                          C.c_void_p(d_weights or None), C.c_void_p(d_sums),
                                                          C.c_void_p(hip_stream or None)),
               "gm_normalize_weights_device")

    def particle_map(self, p: int):
        sx, sy = self.size
        n = np.empty(sx * sy, np.int32)
        v = np.empty(sx * sy, np.int32)
        acc = np.empty(2 * sx * sy, np.float32)
        _check(self.L, self.L.gm_get_particle_map(self.h, p, _fp(n), _fp(v), _fp(acc)), "gm_get_particle_map")
        return n.reshape(sy, sx), v.reshape(sy, sx), acc.reshape(sy, sx, 2)

    def publish(self, p: int) -> np.ndarray:
        sx, sy = self.size
        o = np.empty(sx * sy, np.int8)
        _check(self.L, self.L.gm_publish(self.h, p, _fp(o)), "gm_publish")
        return o.reshape(sy, sx)

    def scores(self):
        s = np.empty(self.P, np.int32)
        h = np.empty(self.P, np.int32)
        f = np.empty(self.P, np.int64)
        _check(self.L, self.L.gm_get_scores(self.h, _fp(s), _fp(h), _fp(f)), "gm_get_scores")
        return s, h, f

    def set_timing(self, on: bool):
        _check(self.L, self.L.gm_set_timing(self.h, 1 if on else 0), "gm_set_timing")

    def kernel_times(self, reset=True):
        ms = C.c_double()
        n = C.c_int64()
        _check(self.L, self.L.gm_get_kernel_times(self.h, C.byref(ms), C.byref(n), 1 if reset else 0),
               "gm_get_kernel_times")
        return ms.value, n.value


def normalize_weights(scores, group=None):
    """Particle weights from the particles' integer scores, across every rank that holds particles:
    w_p = (score_p + 1) / Σ_all (score_q + 1)  (the +1 keeps a particle with no agreeing hit alive).

    The exchange is ONE all-reduce of [Σ(score+1), Σ(score+1)^2] (RCCL on the GPU box, gloo in the
    CPU tests); returns (local weights as float64 tensor, effective sample size of the whole set).
    `scores` is a torch int tensor of this rank's particles (device or CPU)."""
    import torch
    import torch.distributed as dist

    s = scores.to(torch.float64) + 1.0
    red = torch.stack([s.sum(), (s * s).sum()])
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(red, op=dist.ReduceOp.SUM, group=group)
    total, sq = red[0], red[1]
    w = s / total
    neff = (total * total) / sq
    return w, float(neff)


NCCL_UNIQUE_ID_BYTES = 128  # rccl.h


class _UniqueId(C.Structure):
    # ncclUniqueId {char internal[NCCL_UNIQUE_ID_BYTES]}: raw bytes (a random magic + a sockaddr, so it
    # holds NUL bytes) -- an unsigned byte array, never a C string
    _fields_ = [("internal", C.c_uint8 * NCCL_UNIQUE_ID_BYTES)]


def unique_id_bytes(uid: _UniqueId) -> np.ndarray:
    """All NCCL_UNIQUE_ID_BYTES bytes of an ncclUniqueId as uint8 (a c_char array field would stop at the
    first NUL: ctypes reads c_char arrays as C strings)."""
    b = C.string_at(C.addressof(uid), C.sizeof(uid))
    assert len(b) == NCCL_UNIQUE_ID_BYTES
    return np.frombuffer(b, np.uint8).copy()


def unique_id_from_bytes(buf) -> _UniqueId:
    buf = np.ascontiguousarray(buf, np.uint8).reshape(-1)
    if buf.size != NCCL_UNIQUE_ID_BYTES:
        raise Slam2dError(f"ncclUniqueId must be {NCCL_UNIQUE_ID_BYTES} bytes, got {buf.size}")
    uid = _UniqueId()
    C.memmove(C.addressof(uid), buf.tobytes(), NCCL_UNIQUE_ID_BYTES)
    return uid


def exchange_unique_id(uid: _UniqueId | None, world: int, rank: int, bcast) -> _UniqueId:
    """Rank 0's ncclUniqueId on every rank: bcast(uint8[128]) broadcasts rank 0's array (e.g. over
    torch.distributed); every rank checks that all 128 bytes arrived."""
    if world <= 1:
        return uid
    buf = unique_id_bytes(uid) if rank == 0 else np.zeros(NCCL_UNIQUE_ID_BYTES, np.uint8)
    out = np.asarray(bcast(buf), np.uint8).reshape(-1)
    if out.size != NCCL_UNIQUE_ID_BYTES:
        raise Slam2dError(f"unique id broadcast returned {out.size} bytes, expected {NCCL_UNIQUE_ID_BYTES}")
    return unique_id_from_bytes(out)


class RcclComm:
    """An RCCL communicator over the ranks of the job, made the way a C++ host would make one
    (ncclGetUniqueId on rank 0, ncclCommInitRank everywhere); the unique id travels over `bcast`
    (a callable broadcasting a uint8 numpy array from rank 0, e.g. over torch.distributed).  Its
    handle is what gm_normalize_weights_device takes as `nccl_comm`."""

    def __init__(self, world: int, rank: int, bcast=None):
        self._R = C.CDLL("librccl.so.1")
        self._R.ncclGetUniqueId.argtypes = [C.POINTER(_UniqueId)]
        self._R.ncclCommInitRank.argtypes = [C.POINTER(C.c_void_p), C.c_int, _UniqueId, C.c_int]
        self._R.ncclCommDestroy.argtypes = [C.c_void_p]
        self._R.ncclGetErrorString.restype = C.c_char_p
        uid = _UniqueId()
        if rank == 0:
            self._ok(self._R.ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
        uid = exchange_unique_id(uid, int(world), int(rank), bcast)
        h = C.c_void_p()
        self._ok(self._R.ncclCommInitRank(C.byref(h), int(world), uid, int(rank)), "ncclCommInitRank")
        self.handle = h.value

    def _ok(self, rc, what):
        if rc != 0:
            raise Slam2dError(f"{what} failed: {self._R.ncclGetErrorString(rc).decode()}")

    def close(self):
        if self.handle:
            self._R.ncclCommDestroy(C.c_void_p(self.handle))
            self.handle = None
