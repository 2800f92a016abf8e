#!/usr/bin/env python3
"""Build a pricing / A-B variant of the product library from a patched COPY of the sources.

  python tools/build_diag.py <variant> [<variant> ...]     -> creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_<variant>.so

The product sources carry no wrong-result switches: every variant here is a textual patch applied to
a temporary copy of csrc/ (the build fails loudly if a patch no longer applies).  Variants marked
WRONG RESULTS only price a phase of a kernel (tools/ab_bench.sh times them); never ship them.
`python tools/build_diag.py --check` lists variants whose anchors went stale (a CPU test runs it); round 4
removed those of the round-3 kernels it replaced (clk, dwordq, fullstore, mclk, noapply, noapplymath,
nosetup, notiles, seq4acc: see git history before round 4).  The hs_update_kernel variants below price the
round-3 clip kernel (run them with SLAM2D_UPD_KERNEL=clip).

  plain      WRONG RESULTS  hs_update_kernel marks with plain LDS stores instead of atomicMin
  hwexp      WRONG RESULTS  hs_match_kernel uses the hardware exp instead of (float)exp(double)
  gmplain    WRONG RESULTS  gm_compute_kernel walks with plain LDS stores instead of atomicAdd
  gmnowalk   WRONG RESULTS  gm_compute_kernel clips every line to the tile but skips the walk
  nowalk     WRONG RESULTS  hs_update_kernel clips every ray to the tile but skips the Bresenham walk
  plfastatan WRONG RESULTS  pl_icp_kernel uses float atan / atan2 (prices the exact double ones)
  ktnorender WRONG RESULTS  kt_addscans_kernel clears, loads and stores its tiles but renders no item
  lds6       same results   hs_update_kernel with 8.2 KB of unused LDS (8 -> 6 workgroups per CU: occupancy price)
  lds4       same results   hs_update_kernel with 21 KB of unused LDS (4 workgroups per CU)
  frozen     WRONG RESULTS  hs_match_kernel runs no Gauss-Newton iteration (pose = hint): the rays no longer depend
                            on the map, so an update-kernel pricing variant built as frozen__<variant> and timed
                            against frozen alone is not confounded by a drifting match
  ktnoswar   WRONG RESULTS  kt_addscans_kernel dword render writes the kernel bytes without the byte max
  ktnomerge  WRONG RESULTS  kt_build_kernel skips the 64-bit CAS merge of its tile into the match grid
  ktstore    WRONG RESULTS  kt_build_kernel merges with plain stores instead of compare-and-swap
  phase1     same results   hs_match_kernel: workgroups with block id bit 8 set start ~3.6 us late (s_sleep): are
                            the co-resident workgroups' GN steps in lockstep?
  phase2     same results   the same, ~7 us
  noorigin   WRONG RESULTS  hs_update_kernel skips every ray's first 8 free steps (prices the dense cells around
                            the scan origin, where the lanes' atomics hit the same words)
  nohitbit   WRONG RESULTS  hs_update_kernel sets no hit bits (prices the end cells' atomicOr on shared words).
                            CONFOUNDED: with no occupied cells the match drifts, so the rays and the tiles they
                            cover change; a hit-bit word map with <= 4 cells per word timed the same as the
                            32-cell half-row words (round 3), i.e. the atomicOr is not what this variant saves
  seqnochain WRONG RESULTS  hs_match_kernel's chain wave (gn_step_cw, the default) adds one term per chunk (prices
                            the chain adds; the chunk hand-offs and barriers stay)
  chainregs  WRONG RESULTS  hs_match_kernel's chain reads its first 16 terms from LDS and then re-adds the
                            registers it holds (same adds, no further LDS reads: prices the chain's LDS latency)
  noprio     same results   hs_match_kernel's chain wave (gn_step_cw, the default) stays at the default wave priority
  noload     WRONG RESULTS  hs_update_kernel applies its marks to zeros instead of loading the marked quads (prices the
                            apply's load latency, exposed once per tile when the raster before it is short)
  nostore    WRONG RESULTS  hs_update_kernel computes the apply but stores nothing (prices the write traffic)
  noord      WRONG RESULTS  hs_update_kernel stores no update ordinal (log-odds exact: prices the ordinal plane's stores;
                            round 5's noidx / idx16 priced the 32-bit plane before it: profiles/r05/INDEX.md)
  ordbm      WRONG RESULTS  hs_update_kernel stores, per wave and marked tile, its lanes' mark + hit bits (one 2-B store per
                            lane, 128 B per wave) and a 16-B header from lane 0 instead of the ordinals (prices a bitmap
                            log of the ordinal plane, round-6 VERDICT item 1; the fold kernel is priced separately)
  ordbm2     WRONG RESULTS  ordbm without the header store and the any-mark test: every thread of a tile with marks stores
                            its 2-B bit word (the floor of a bitmap log's store cost in the update)
  valu100    same results   hs_update_kernel issues 100 extra independent v_add_f32 per tile iteration per wave (prices the
                            kernel's sensitivity to VALU issue: ~+40 % of its VALU instructions)
  ordfull    WRONG RESULTS  hs_update_kernel stores every marked quad's four ordinals in one 8-B store, unmarked cells
                            included (prices per-cell 2-B stores against one store per quad)
  uclk       same results   hs_update_kernel's waves sum s_memtime cycles per tile-loop phase (raster, load/store wait,
                            apply, barrier, mark read) into the diagnostic stamps: tools/clk_update.py reads them
  nobar      WRONG RESULTS  hs_update_kernel without the per-tile barrier (each wave reads its quads' marks when its own
                            raster is done; races with the other waves' rasters): prices the four waves' coupling
  mclk       same results   hs_match_kernel's chain wave sums s_memtime cycles per Gauss-Newton step: step start -> chain
                            start (gathers, conversions, chunk 0), the chain, its end -> the next step (solve, broadcast);
                            tools/clk_match.py reads them
  mclkbar    same results   mclk, with stamp 3 = the chain wave's cycles inside its chunk barriers (chunks 1..)
  cheapprob  WRONG RESULTS  cell_prob is one multiply-add instead of exp + division (prices the match's probability
                            conversions: their VALU and their place on the per-stream path)
  mlds4      same results   hs_match_kernel with 1.2 KB of unused LDS (5 -> 4 workgroups per CU: is the chain's
                            contention worth a fifth of the streams per CU?)
  mlds3      same results   hs_match_kernel with 12 KB of unused LDS (4 -> 3 workgroups per CU: prices the match's
                            streams per CU)
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
    "hwexp": [(K, "    float odds = sdm_expf_tab(l, s_exptab);", "    float odds = __expf(l);")],
    "gmplain": [("gmapping_kernels.hip", "        atomicAdd(reinterpret_cast<unsigned *>(pc), 1u); /* visits++ (:227-234) */ \\\n",
                 "        *reinterpret_cast<volatile unsigned *>(pc) = 1u;                             \\\n")],
    "gmnowalk": [("gmapping_kernels.hip", "            if (GM_PRICE == 3) return;\n", "            return;\n")],  # (= GM_PRICE=3)
    "plfastatan": [("plicp_kernels.hip", '#include "detmath.h"\n',
                    '#include "detmath.h"\n#define sdm_atan2(y, x) ((double)atan2f((float)(y), (float)(x)))\n'
                    '#define sdm_atan(x) ((double)atanf((float)(x)))\n')],
    "nowalk": [(K, "                    if ((int)!met | (int)(lo_i > hi_i)) continue;\n                    anyv = 1u;\n",
                "                    if ((int)!met | (int)(lo_i > hi_i)) continue;\n                    anyv = 1u;\n                    continue;\n")],
    "ktnorender": [("karto_kernels.hip", "kt_render_items_dw(tileb, sitem, c0, c1,", "kt_render_items_dw(tileb, sitem, c0, c0,")],
    "lds6": [("hector_capi.hip", "UPD_GROUP_WORDS * (size_t)fan_groups(c->max_points));\n}",
              "UPD_GROUP_WORDS * (size_t)fan_groups(c->max_points) + 2100);\n}")],
    "lds4": [("hector_capi.hip", "UPD_GROUP_WORDS * (size_t)fan_groups(c->max_points));\n}",
              "UPD_GROUP_WORDS * (size_t)fan_groups(c->max_points) + 5430);\n}")],
    "ktnomerge": [("karto_kernels.hip", "    for (int t0 = lane; t0 < nw; t0 += 64 * 8) {\n        unsigned long long want[8], old[8];",
                   "    if (nw > 0) return true;\n    for (int t0 = lane; t0 < nw; t0 += 64 * 8) {\n        unsigned long long want[8], old[8];")],
    "ktstore": [("karto_kernels.hip", "                old[u] = atomicCAS(gw + wbase + r * wsw + q, 0ull, want[u]);",
                 "                gw[wbase + r * wsw + q] = want[u];")],
    "phase1": [(K, "    load_exptab();\n    if (!fused) __syncthreads();",
                "    if ((blockIdx.x >> 8) & 1) __builtin_amdgcn_s_sleep(127);\n    load_exptab();\n    if (!fused) __syncthreads();")],
    "phase2": [(K, "    load_exptab();\n    if (!fused) __syncthreads();",
                "    if ((blockIdx.x >> 8) & 1) { __builtin_amdgcn_s_sleep(127); __builtin_amdgcn_s_sleep(127); }\n"
                "    load_exptab();\n    if (!fused) __syncthreads();")],
    "noorigin": [(K, "                    if ((int)!met | (int)(lo_i > hi_i)) continue;\n",
                  "                    if (lo_i < 8) lo_i = 8;\n                    if (!met | (lo_i > hi_i)) continue;\n")],
    "nohitbit": [(K, "                    atomicOr(&hitb[c >> 5], 1u << (c & 31));\n", "                    (void)c;\n")],
    "seqnochain": [(K, "                run = seq_chain_t<CW_STRIDE>(seqT + (CW_BUFS == 2 ? (j & 1) * CW_BUF : 0), lane, min(CW_PTS, n - j * CW_PTS),\n"
                       "                                             run);\n",
                    "                run = run + seqT[lane * CW_STRIDE];\n")],
    "frozen": [(K, "            for (int it = 0; it <= iters; ++it) {\n                if (in_regs) {",
                "            for (int it = 0; it <= iters && false; ++it) {\n                if (in_regs) {")],
    "chainregs": [(K, "            b0 = row[i]; b1 = row[i + 1]; b2 = row[i + 2]; b3 = row[i + 3];\n",
                   "            b0 = a0; b1 = a1; b2 = a2; b3 = a3;\n"),
                  (K, "            a0 = row[i + 4]; a1 = row[i + 5]; a2 = row[i + 6]; a3 = row[i + 7];\n", "")],
    "noprio": [(K, "        // (the workgroup's critical path issues ahead of co-resident workgroups' waves)\n        __builtin_amdgcn_s_setprio(3);\n",
                "        // (the workgroup's critical path issues ahead of co-resident workgroups' waves)\n        __builtin_amdgcn_s_setprio(0);\n")],
    "mlds3": [(K, "    __shared__ float s_pose[2][POSE_WORDS];                             // a step's result, by parity\n",
               "    __shared__ float s_pose[2][POSE_WORDS];                             // a step's result, by parity\n"
               "    __shared__ float s_pad[3000];\n    if (stream_begin < 0) s_pad[threadIdx.x] = 1.0f;\n")],
    "mlds4": [(K, "    __shared__ float s_pose[2][POSE_WORDS];                             // a step's result, by parity\n",
               "    __shared__ float s_pose[2][POSE_WORDS];                             // a step's result, by parity\n"
               "    __shared__ float s_pad[300];\n    if (stream_begin < 0) s_pad[threadIdx.x] = 1.0f;\n")],
    "noload": [(K, "                    if (mk) ql[j] = *reinterpret_cast<const float4 *>(pend_tl + (unsigned)upd_off(row, c4, g.tiles_x));\n",
                "                    if (mk) ql[j] = make_float4(0.0f, 0.0f, 0.0f, (float)row);\n")],
    "nostore": [(K, "__device__ __forceinline__ void upd_store(float4 *p, float4 v)\n{\n#if S2D_NT_STORE",
                 "__device__ __forceinline__ void upd_store(float4 *p, float4 v)\n{\n    if (v.x == 1234.5f) *p = v;\n    return;\n#if S2D_NT_STORE"),
                (K, "__device__ __forceinline__ void upd_store(int4 *p, int4 v)\n{\n#if S2D_NT_STORE",
                 "__device__ __forceinline__ void upd_store(int4 *p, int4 v)\n{\n    if (v.x == 1234) *p = v;\n    return;\n#if S2D_NT_STORE"),
                (K, "__device__ __forceinline__ void upd_store(int *p, int v)\n{\n#if S2D_NT_STORE",
                 "__device__ __forceinline__ void upd_store(int *p, int v)\n{\n    if (v == 1234) *p = v;\n    return;\n#if S2D_NT_STORE")],
    "noord": [(K, "                if (qb_all(mb)) {\n                    *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));\n                } else {\n#pragma unroll\n                    for (int c = 0; c < 4; ++c)\n                        if (qb_cell(mb, c)) tu[ou + (unsigned)c] = (unsigned short)uv[c];\n                }\n", "")],
    "ordbm": [(K, "                if (qb_all(mb)) {\n                    *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));\n                } else {\n#pragma unroll\n                    for (int c = 0; c < 4; ++c)\n                        if (qb_cell(mb, c)) tu[ou + (unsigned)c] = (unsigned short)uv[c];\n                }\n", "                (void)uv;\n"),
              (K, "                touched += qb_count(mb);\n            }\n            pend_tl = nullptr;\n",
               "                touched += qb_count(mb);\n            }\n            {\n                unsigned bm = 0u;\n#pragma unroll\n"
               "                for (int j = 0; j < UPD_QUADS; ++j) {\n                    const unsigned u = ~qb[j] & QB_UNMASK;\n"
               "                    const unsigned mk = ((u >> 7) & 1u) | ((u >> 14) & 2u) | ((u >> 21) & 4u) | (u >> 28);\n"
               "                    bm |= (mk | (qb_hits(qb[j]) << 3)) << (8 * j);\n                }\n"
               "                if (__any(bm != 0u)) {\n                    tu[qtid] = (unsigned short)bm;\n"
               "                    if (lane == 0) *reinterpret_cast<uint4 *>(&pend_tl[ORD_OFF + 512 + 4 * (qtid >> 6)]) = "
               "make_uint4(mark_free, (unsigned)(size_t)pend_tl, 0u, 0u);\n                }\n            }\n            pend_tl = nullptr;\n")],
    "ordbm2": [(K, "                if (qb_all(mb)) {\n                    *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));\n                } else {\n#pragma unroll\n                    for (int c = 0; c < 4; ++c)\n                        if (qb_cell(mb, c)) tu[ou + (unsigned)c] = (unsigned short)uv[c];\n                }\n", "                (void)uv;\n"),
               (K, "                touched += qb_count(mb);\n            }\n            pend_tl = nullptr;\n",
                "                touched += qb_count(mb);\n            }\n            {\n                unsigned bm = 0u;\n#pragma unroll\n"
                "                for (int j = 0; j < UPD_QUADS; ++j) {\n                    const unsigned u = ~qb[j] & QB_UNMASK;\n"
                "                    const unsigned mk = ((u >> 7) & 1u) | ((u >> 14) & 2u) | ((u >> 21) & 4u) | (u >> 28);\n"
                "                    bm |= (mk | (qb_hits(qb[j]) << 3)) << (8 * j);\n                }\n"
                "                tu[qtid] = (unsigned short)(bm | (mark_free << 16));\n            }\n            pend_tl = nullptr;\n")],
    "valu100": [(K, "        const int X0 = tx * TILE, Y0 = ty * UPD_TH;\n",
                 "        const int X0 = tx * TILE, Y0 = ty * UPD_TH;\n"
                 "        { float dmy_; asm volatile(\".rept 100\\n\\tv_add_f32 %0, %1, %2\\n\\t.endr\" : \"=v\"(dmy_) : \"v\"((float)X0), \"v\"((float)Y0)); }\n")],
    "ordfull": [(K, "                if (qb_all(mb)) {\n                    *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));\n                } else {\n#pragma unroll\n                    for (int c = 0; c < 4; ++c)\n                        if (qb_cell(mb, c)) tu[ou + (unsigned)c] = (unsigned short)uv[c];\n                }\n",
                 "                *reinterpret_cast<uint2 *>(&tu[ou]) = make_uint2(uv[0] | (uv[1] << 16), uv[2] | (uv[3] << 16));\n")],
    "uclk": [(K, "    for (int ii = 0; ii <= my_tiles; ++ii) {\n        const int i = __builtin_amdgcn_readfirstlane(ii);  // uniform (the compiler had put it in a VGPR)\n        const int qtid = tid;",
              "    unsigned long long u_r = 0, u_w = 0, u_a = 0, u_b = 0, u_m = 0, u_t = __builtin_amdgcn_s_memtime();\n"
              "#define UCLK(acc) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); acc += t_ - u_t; u_t = t_; } while (0)\n"
              "    for (int ii = 0; ii <= my_tiles; ++ii) {\n        UCLK(u_m);\n        const int i = __builtin_amdgcn_readfirstlane(ii);  // uniform (the compiler had put it in a VGPR)\n        const int qtid = tid;"),
             (K, "        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)\n",
              "        UCLK(u_r);\n        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)\n        UCLK(u_w);\n"),
             (K, "            lds_barrier();  // tile i's marks complete\n            if (s_any[buf] == (unsigned)(i + 1)) {\n                // thread owns quads",
              "            UCLK(u_a);\n            lds_barrier();  // tile i's marks complete\n            UCLK(u_b);\n            if (s_any[buf] == (unsigned)(i + 1)) {\n                // thread owns quads"),
             (K, "\n    for (int off = 32; off >= 1; off >>= 1) touched += __shfl_xor(touched, off, 64);\n",
              "\n    UCLK(u_m);\n    if (lane == 0) {\n        atomicAdd(&g_stamps[0], u_r); atomicAdd(&g_stamps[1], u_w); atomicAdd(&g_stamps[2], u_a);\n"
              "        atomicAdd(&g_stamps[3], u_b); atomicAdd(&g_stamps[4], u_m); atomicAdd(&g_stamps[5], 1ull);\n"
              "        atomicAdd(&g_stamps[6], (unsigned long long)my_tiles);\n    }\n"
              "    for (int off = 32; off >= 1; off >>= 1) touched += __shfl_xor(touched, off, 64);\n")],
    "nobar": [(K, "            lds_barrier();  // tile i's marks complete\n            if (s_any[buf] == (unsigned)(i + 1)) {\n                // thread owns quads",
               "            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only: no barrier\n            if (s_any[buf] == (unsigned)(i + 1)) {\n                // thread owns quads")],
    "mclk": [(K, "template <int NP, bool BIG>\n__device__ __forceinline__ void gn_step_cw(",
              "extern __device__ unsigned long long g_stamps[8];\n__shared__ unsigned long long s_mk[8];\n"
              "template <int NP, bool BIG>\n__device__ __forceinline__ void gn_step_cw("),
             (K, "    if (S2D_PRECHAIN_PRIO) __builtin_amdgcn_s_setprio(S2D_PRECHAIN_PRIO);\n    if (wave != cw) {\n        // the moved points' neighbourhoods",
              "    unsigned long long mk_t0 = __builtin_amdgcn_s_memtime(), mk_t1 = 0, mk_t2 = 0, mk_pa = 0, mk_pb = 0, mk_pc = 0; bool mk_big = false;\n"
              "    if (S2D_PRECHAIN_PRIO) __builtin_amdgcn_s_setprio(S2D_PRECHAIN_PRIO);\n    if (wave != cw) {\n        // the moved points' neighbourhoods"),
             (K, "            lds_barrier();\n            if (lane < 9)\n                run = seq_chain_t<CW_STRIDE>(",
              "            lds_barrier();\n            if (j == 0) mk_t1 = __builtin_amdgcn_s_memtime();\n            if (lane < 9)\n                run = seq_chain_t<CW_STRIDE>("),
             (K, "                                             run);\n        }\n    }\n    float *sp = s_pose[parity];\n    if (wave == cw) {\n        float s[9], H[9];",
              "                                             run);\n        }\n        mk_t2 = __builtin_amdgcn_s_memtime();\n    }\n    float *sp = s_pose[parity];\n    if (wave == cw) {\n        float s[9], H[9];"),
             (K, "    __syncthreads();\n    // (H stays in s_pose, read once at the level's end)\n    est[0] = sp[0];\n    est[1] = sp[1];\n    est[2] = sp[2];\n    cs = sp[3];\n    sn = sp[4];\n}\n\nconstexpr int MATCH_REG_PTS",
              "    if (wave == cw && lane == 0) {\n        const unsigned long long mk_t3 = __builtin_amdgcn_s_memtime();\n"
              "        s_mk[0] += mk_t1 - mk_t0; s_mk[1] += mk_t2 - mk_t1; s_mk[2] += mk_t3 - mk_t2;\n    }\n"
              "    if (wave != cw && pt == 0) { s_mk[4] += mk_pa - mk_t0; s_mk[5] += mk_pb - mk_pa; s_mk[6] += mk_pc - mk_pb; if (mk_big) s_mk[7] += mk_pb - mk_pa; }\n"
              "    __syncthreads();\n    // (H stays in s_pose, read once at the level's end)\n    est[0] = sp[0];\n    est[1] = sp[1];\n    est[2] = sp[2];\n    cs = sp[3];\n    sn = sp[4];\n}\n\nconstexpr int MATCH_REG_PTS"),
             (K, "        if (first) {\n            // a level's first step",
              "        mk_pa = __builtin_amdgcn_s_memtime();\n        if (first) {\n            // a level's first step"),
             (K, "        lds_barrier();\n    }\n    if (wave != cw) {\n        // chunk j = slot j",
              "        lds_barrier();\n    }\n    mk_pb = __builtin_amdgcn_s_memtime();\n    if (wave != cw) {\n        // chunk j = slot j"),
             (K, "            lds_barrier();  // chunk j stored (two buffers: and the chain wave is done with chunk j - 1)\n",
              "            lds_barrier();  // chunk j stored (two buffers: and the chain wave is done with chunk j - 1)\n            if (j == 0) mk_pc = __builtin_amdgcn_s_memtime();\n"),
             (K, "        const int c0 = s_mcnt[0], c1 = s_mcnt[1], tot = c0 + c1 + s_mcnt[2];\n",
              "        const int c0 = s_mcnt[0], c1 = s_mcnt[1], tot = c0 + c1 + s_mcnt[2];\n        mk_big = tot >= 512;\n        if (tid == 0 && mk_big) s_mk[3] += 1ull;\n"),
             (K, "    load_exptab();\n    if (!fused) __syncthreads();",
              "    if (threadIdx.x < 8) s_mk[threadIdx.x] = 0ull;\n    load_exptab();\n    if (!fused) __syncthreads();"),
             (K, "    clk_stamp(geom.clk, 0, false);\n    if (threadIdx.x != 0) return;",
              "    clk_stamp(geom.clk, 0, false);\n    if (threadIdx.x == 0) for (int k = 0; k < 8; ++k) atomicAdd(&g_stamps[k], s_mk[k]);\n    if (threadIdx.x != 0) return;")],
    # mclk with stamp 3 = the chain wave's cycles inside its chunk barriers (chunks 1..), instead of the count of
    # steps with >= 512 misses (tools/clk_match.py with CLK_BAR=1)
    "mclkbar": None,
    "cheapprob": [(K, "    float odds = sdm_expf_tab(l, s_exptab);\n    return __fdiv_rn(odds, odds + 1.0f);",
                   "    return l * 0.25f + 0.5f;")],
    "ktnoswar": [("karto_kernels.hip", "    return b ^ ((a ^ b) & (t - (t >> 7)));", "    return b | (t & 0u);")],
}


def _mclkbar():
    out = []
    for fname, a, b in PATCHES["mclk"]:
        if "mk_big = tot >= 512;" in b:
            b = b.replace("        if (tid == 0 && mk_big) s_mk[3] += 1ull;\n", "")
        out.append((fname, a, b))
    out.append((K, "            if (CW_BUFS == 1 && (!CW_SHARE || j > 0)) lds_barrier();\n            lds_barrier();\n"
                   "            if (j == 0) mk_t1 = __builtin_amdgcn_s_memtime();\n",
                "            const unsigned long long mk_b0 = __builtin_amdgcn_s_memtime();\n"
                "            if (CW_BUFS == 1 && (!CW_SHARE || j > 0)) lds_barrier();\n            lds_barrier();\n"
                "            if (j == 0) mk_t1 = __builtin_amdgcn_s_memtime();\n"
                "            else if (lane == 0) s_mk[3] += __builtin_amdgcn_s_memtime() - mk_b0;\n"))
    return out


PATCHES["mclkbar"] = _mclkbar()


def build(variant: str) -> str:
    parts = variant.split("__")  # a__b: both patch lists (e.g. frozen__noapply)
    for v in parts:
        if v not in PATCHES:
            raise SystemExit(f"unknown variant {v!r}; known: {', '.join(sorted(PATCHES))}")
    tmp = tempfile.mkdtemp()
    try:
        src = os.path.join(tmp, "creating-2d-laser-slam-from-scratch_amd", "csrc")
        shutil.copytree(os.path.join(PKG, "csrc"), src)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
        for fname, old, new in [p for v in parts for p in PATCHES[v]]:
            p = os.path.join(src, fname)
            text = open(p).read()
            if text.count(old) != 1:
                raise SystemExit(f"variant {variant}: patch anchor not found exactly once in {fname}: {old[:60]!r}")
            open(p, "w").write(text.replace(old, new))
        out = os.path.join(PKG, "lib", "ab", f"libslam2d_{variant}.so")
        subprocess.check_call(["make", "-s", "-C", src, f"OUT={out}"])
        return out
    finally:
        shutil.rmtree(tmp)


def check() -> list:
    """Variants whose patch anchors no longer occur exactly once in the sources (tests/test_host_cpu.py)."""
    bad = []
    for v, patches in sorted(PATCHES.items()):
        text = {}  # the variant's patches apply in order, each to the text the previous ones left (as build() does)
        for fname, old, new in patches:
            if fname not in text:
                with open(os.path.join(PKG, "csrc", fname)) as f:
                    text[fname] = f.read()
            if text[fname].count(old) != 1:
                bad.append(v)
                break
            text[fname] = text[fname].replace(old, new)
    return bad


if __name__ == "__main__":
    if sys.argv[1:] == ["--check"]:
        bad = check()
        print("stale variants:", bad or "none")
        sys.exit(1 if bad else 0)
    for v in sys.argv[1:]:
        print("built", build(v))
