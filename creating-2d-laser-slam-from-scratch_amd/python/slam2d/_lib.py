"""ctypes loader for the MI355X product library (lib/libslam2d.so, built from csrc/ for gfx950).

There is no CPU fallback: if the library is missing or no HIP device is present, the product API
raises.  torch is imported first (when available) so that the library binds to the same HIP
runtime instance torch already loaded (both carry SONAME libamdhip64.so.7), which lets device
pointers and hipStream_t handles from torch tensors be passed through the C-ABI.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(PKG_ROOT, "csrc")
LIB_PATH = os.environ.get("SLAM2D_LIB") or os.path.join(PKG_ROOT, "lib", "libslam2d.so")

_f, _i, _p = C.c_float, C.c_int, C.c_void_p
_LIB = None


class Slam2dError(RuntimeError):
    pass


def build(force: bool = False) -> str:
    """Compile csrc/ for gfx950 with hipcc (make -C csrc)."""
    if force and os.path.exists(LIB_PATH):
        os.remove(LIB_PATH)
    subprocess.check_call(["make", "-s", "-C", CSRC])
    return LIB_PATH


def _declare(L):
    P = C.POINTER
    L.hs_version.restype = C.c_char_p
    if hasattr(L, "hs_source_id"):
        L.hs_source_id.restype = C.c_char_p
    L.hs_last_error.restype = C.c_char_p
    L.hs_create.argtypes = [P(_p), _i, _f, _i, _i, _f, _f, _i, _i]
    L.hs_destroy.argtypes = [_p]
    L.hs_reset.argtypes = [_p]
    L.hs_set_update_factors.argtypes = [_p, _f, _f]
    L.hs_set_map_update_thresholds.argtypes = [_p, _f, _f]
    L.hs_get_scale_to_map.argtypes = [_p, P(_f)]
    L.hs_get_map_levels.argtypes = [_p, P(_i)]
    L.hs_get_map_info.argtypes = [_p, _i, P(_i), P(_i), P(_f), _p]
    L.hs_update.argtypes = [_p, _i, _p, _i, _f, _f, _p, _i, _p, _p, P(_i)]
    L.hs_match.argtypes = [_p, _i, _p, _i, _f, _f, _p, _p, _p]
    L.hs_update_by_scan.argtypes = [_p, _i, _p, _i, _f, _f, _p]
    L.hs_get_last_pose.argtypes = [_p, _i, _p, _p]
    L.hs_get_map.argtypes = [_p, _i, _i, _p, _p, _p, P(_i)]
    L.hs_set_map.argtypes = [_p, _i, _i, _p, _p]
    L.hs_step_batch_device.argtypes = [_p, _i, _i, _p, _i, _p, _p, _p, _p]
    L.hs_get_poses.argtypes = [_p, _p, _p, _p, _p]
    L.hs_get_counters.argtypes = [_p, _p, _i]
    L.hs_get_queue_stats.argtypes = [_p, _p, _i]
    if hasattr(L, "hs_get_diag_stamps"):  # (A/B runs may load libraries built before this diagnostic existed)
        L.hs_get_diag_stamps.argtypes = [_p, _p, _i]
    L.hs_get_device_buffers.argtypes = [_p, P(_p), P(C.c_size_t), P(C.c_size_t)]
    if hasattr(L, "hs_flush_ordinals"):  # (A/B runs may load libraries built before round 6)
        L.hs_flush_ordinals.argtypes = [_p, _p]
    L.hs_set_pose_log.argtypes = [_p, _p, _i, _i]
    L.hs_set_pose_log_slots.argtypes = [_p, _p, _p, _i, _i]
    L.hs_run_ranges_device.argtypes = [_p, _i, _p, _i, C.c_size_t, _p]
    L.hs_get_stream.restype = _p
    L.hs_get_stream.argtypes = [_p]
    L.hs_set_timing.argtypes = [_p, _i]
    L.hs_get_kernel_times.argtypes = [_p, _p, _p, _i]
    L.hs_set_clock_probe.argtypes = [_p, _i]
    L.hs_get_clock_probe.argtypes = [_p, _p, _i]
    L.hs_default_laser.restype = None
    L.hs_default_laser.argtypes = [_p, _i, _f, _f]
    L.hs_set_laser.argtypes = [_p, _p, _p]
    L.hs_ingest_batch_device.argtypes = [_p, _i, _p, _i, _p, _i, _p, _p, _p]
    L.hs_step_ranges_batch_device.argtypes = [_p, _i, _i, _p, _i, _p, _p]
    L.hs_update_ranges.argtypes = [_p, _i, _p, _p, _p, P(_i)]
    L.hs_set_reduction_order.argtypes = [_p, _i]
    L.hs_get_reduction_order.argtypes = [_p, P(_i)]
    # GMapping particle path (include/slam2d/gmapping.h)
    D = C.c_double
    L.gm_version.restype = C.c_char_p
    L.gm_last_error.restype = C.c_char_p
    L.gm_create.argtypes = [P(_p), _i, _i, D, D, D, D, D, D, D]
    L.gm_destroy.argtypes = [_p]
    L.gm_reset.argtypes = [_p]
    L.gm_set_beams.argtypes = [_p, _p, _p, _i]
    L.gm_set_occ_thresh.argtypes = [_p, D]
    L.gm_get_map_size.argtypes = [_p, P(_i), P(_i)]
    L.gm_compute_maps.argtypes = [_p, _p, _p, _i]
    L.gm_compute_maps_device.argtypes = [_p, _i, _i, _p, _p, _i, _p, _p]
    L.gm_get_particle_map.argtypes = [_p, _i, _p, _p, _p]
    L.gm_publish.argtypes = [_p, _i, _p]
    L.gm_get_scores.argtypes = [_p, _p, _p, _p]
    L.gm_set_timing.argtypes = [_p, _i]
    L.gm_get_kernel_times.argtypes = [_p, _p, _p, _i]
    L.gm_normalize_weights_device.argtypes = [_p, _p, _p, _i, _p, _p, _p]


def lib() -> C.CDLL:
    """Load lib/libslam2d.so (fails loudly if it was not built)."""
    global _LIB
    if _LIB is None:
        try:  # share torch's HIP runtime instance if torch is present
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise Slam2dError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() or `make -C {CSRC}`")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        _LIB = L
    return _LIB


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().hs_last_error().decode(errors="replace")
        raise Slam2dError(f"{what} failed with code {rc}: {msg}")


def source_id_of_tree() -> str:
    """16 hex digits of sha256 over the Hector kernel sources in csrc/ (the Makefile's SRC_HASH)."""
    import hashlib

    h = hashlib.sha256()
    for name in ("hector_kernels.hip", "hector_capi.hip", "hector_internal.h", "detmath.h"):
        try:
            with open(os.path.join(CSRC, name), "rb") as f:
                h.update(f.read())
        except OSError:
            return ""
    return h.hexdigest()[:16]


def source_id_of_library() -> str:
    """The source hash compiled into the loaded library (hs_source_id; "" for a library built before it)."""
    L = lib()
    return L.hs_source_id().decode() if hasattr(L, "hs_source_id") else ""


def check_library_matches_tree() -> str:
    """Raise when the loaded library was built from other Hector sources than csrc/ holds; return the id."""
    built, tree = source_id_of_library(), source_id_of_tree()
    if tree and built != tree:
        raise Slam2dError(f"{LIB_PATH} was built from Hector sources {built}, csrc/ holds {tree}: rebuild it "
                          f"(__graft_entry__.build())")
    return built


def exported_symbols() -> list[str]:
    """Dynamic symbols the library exports (nm -D), for the ABI test."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB_PATH], text=True)
    return sorted({ln.split()[-1] for ln in out.splitlines() if ln.strip()})
