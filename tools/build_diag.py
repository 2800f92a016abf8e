#!/usr/bin/env python3
"""Build a pricing / A-B variant of the product library from a patched COPY of the sources.

  python tools/build_diag.py <variant> [<variant> ...]     -> creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_<variant>.so

The product sources carry no wrong-result switches: every variant here is a textual patch applied to
a temporary copy of csrc/ (the build fails loudly if a patch no longer applies).  Variants marked
WRONG RESULTS only price a phase of a kernel (tools/ab_bench.sh times them); never ship them.

  plain      WRONG RESULTS  hs_update_kernel marks with plain LDS stores instead of atomicMin
  noapply    WRONG RESULTS  hs_update_kernel skips the apply phase (no global loads / stores)
  hwexp      WRONG RESULTS  hs_match_kernel uses the hardware exp instead of (float)exp(double)
  gmplain    WRONG RESULTS  gm_compute_kernel walks with plain LDS stores instead of atomicAdd
  gmnowalk   WRONG RESULTS  gm_compute_kernel clips every line to the tile but skips the walk
  nowalk     WRONG RESULTS  hs_update_kernel clips every ray to the tile but skips the Bresenham walk
  nosetup    WRONG RESULTS  hs_update_kernel keeps the fan-group culling of every tile, skips every ray
  noraster   WRONG RESULTS  hs_update_kernel skips the raster loop (tile loop skeleton: clear, barriers)
  visits2    same results   as visits: visits, visits with no walking lane, walking lanes, lanes that
                            passed the ray-vs-tile box test (set up a walk)
  visits     same results   hs_update_kernel counts, per (tile, fan group) visit, the lanes with steps,
                            the steps and the wave's longest walk into g_stamps[0..3]
                            (hs_get_queue_stats out[4..7]; tools/diag_update.py prints them)
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "creating-2d-laser-slam-from-scratch_amd")
K = "hector_kernels.hip"

PATCHES = {
    "plain": [(K, "__device__ __forceinline__ void upd_mark(unsigned *p, unsigned ev) { atomicMin(p, ev); }",
               "__device__ __forceinline__ void upd_mark(unsigned *p, unsigned ev) "
               "{ *reinterpret_cast<volatile unsigned *>(p) = ev; }")],
    "noapply": [(K, "        if (pend_tl) {\n", "        if (pend_tl && false) {\n")],
    "hwexp": [(K, "    float odds = sdm_expf(l);", "    float odds = __expf(l);")],
    "gmplain": [("gmapping_kernels.hip", "        atomicAdd(reinterpret_cast<unsigned *>(pc), 1u); /* visits++ (:227-234) */ \\\n",
                 "        *reinterpret_cast<volatile unsigned *>(pc) = 1u;                             \\\n")],
    "gmnowalk": [("gmapping_kernels.hip", "            int i = 0;\n#define GM_WSTEP", "            int i = steps;\n#define GM_WSTEP")],
    "nowalk": [(K, "                if (scnt <= 0) continue;\n", "                continue;\n")],
    "nosetup": [(K, "                if (gx1 < X0 || gx0 >= X1 || gy1 < Y0 || gy0 >= Y1) continue;\n",
                 "                if (gx1 < X0 || gx0 >= X1 || gy1 < Y0 || gy0 >= Y1) continue;\n                continue;\n")],
    "noraster": [(K, "                const int4 gb = gbox[b0 >> 6];\n", "                if (b0 >= 0) break;\n                const int4 gb = gbox[b0 >> 6];\n")],
    "visits2": [(K, "                int scnt = 0;           // free steps of this beam inside the tile\n",
                 "                int scnt = 0;           // free steps of this beam inside the tile\n                bool dsu = false;\n"),
                (K, "                        w = ray_walk(x0, y0, x1, y1);\n",
                 "                        dsu = true;\n                        w = ray_walk(x0, y0, x1, y1);\n"),
                (K, "                if (scnt <= 0) continue;\n",
                 "                {\n"
                 "                    const unsigned long long am = __ballot(scnt > 0), ad = __ballot(dsu);\n"
                 "                    if (lane == 0) {\n"
                 "                        atomicAdd(&g_stamps[0], 1ull);\n"
                 "                        atomicAdd(&g_stamps[1], am ? 0ull : 1ull);\n"
                 "                        atomicAdd(&g_stamps[2], (unsigned long long)__popcll(am));\n"
                 "                        atomicAdd(&g_stamps[3], (unsigned long long)__popcll(ad));\n"
                 "                    }\n"
                 "                }\n"
                 "                if (scnt <= 0) continue;\n")],
    "visits": [(K, "                if (scnt <= 0) continue;\n",
                "                {\n"
                "                    const unsigned long long am = __ballot(scnt > 0);\n"
                "                    int mx = scnt, sm = scnt;\n"
                "                    for (int off = 32; off >= 1; off >>= 1) {\n"
                "                        mx = max(mx, __shfl_xor(mx, off, 64));\n"
                "                        sm += __shfl_xor(sm, off, 64);\n"
                "                    }\n"
                "                    if (lane == 0) {\n"
                "                        atomicAdd(&g_stamps[0], 1ull);\n"
                "                        atomicAdd(&g_stamps[1], (unsigned long long)__popcll(am));\n"
                "                        atomicAdd(&g_stamps[2], (unsigned long long)sm);\n"
                "                        atomicAdd(&g_stamps[3], (unsigned long long)mx);\n"
                "                    }\n"
                "                }\n"
                "                if (scnt <= 0) continue;\n")],
}


def build(variant: str) -> str:
    if variant not in PATCHES:
        raise SystemExit(f"unknown variant {variant!r}; known: {', '.join(sorted(PATCHES))}")
    tmp = tempfile.mkdtemp()
    try:
        src = os.path.join(tmp, "creating-2d-laser-slam-from-scratch_amd", "csrc")
        shutil.copytree(os.path.join(PKG, "csrc"), src)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
        for fname, old, new in PATCHES[variant]:
            p = os.path.join(src, fname)
            text = open(p).read()
            if text.count(old) != 1:
                raise SystemExit(f"variant {variant}: patch anchor not found exactly once in {fname}: {old[:60]!r}")
            open(p, "w").write(text.replace(old, new))
        out = os.path.join(PKG, "lib", f"libslam2d_{variant}.so")
        subprocess.check_call(["make", "-s", "-C", src, f"OUT={out}"])
        return out
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    for v in sys.argv[1:]:
        print("built", build(v))
