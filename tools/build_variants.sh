#!/bin/bash
# Compile-time A/B variants of the product library (same sources, other -D switches) next to libslam2d.so:
#   th64  ring update kernel (opt-in, SLAM2D_UPD_KERNEL=ring) with 64-row tiles and 512-thread workgroups
#   cw2   chain-wave match with two term buffers (S2D_CW_BUFS=2: 38 KB of LDS, 4 workgroups per CU)
#   r3m   round 3's match chain (S2D_MATCH_CW=0)
#   noaf  no apply fast path (S2D_APPLY_FAST=0)
#   nt    non-temporal stores in the update apply (S2D_NT_STORE=1)
#   oct   whole-sector log-odds stores in the update apply (S2D_OCTET=1)
#   oct2  whole-sector stores in both planes (S2D_OCTET=2; 6 workgroups per CU for the extra registers)
#   wedge fan groups culled per tile by the cone of their rays as well as their box (S2D_WEDGE=1)
#   batch  fan-group cull batched over a wave's next tiles (S2D_CULL_BATCH=1); batchw: with the cone cull
set -e
cd "$(dirname "$0")/../creating-2d-laser-slam-from-scratch_amd/csrc"
make -s
make -s OUT=../lib/libslam2d_th64.so EXTRA=-DS2D_RING_TH=64
make -s OUT=../lib/libslam2d_cw2.so EXTRA=-DS2D_CW_BUFS=2
make -s OUT=../lib/libslam2d_r3m.so EXTRA=-DS2D_MATCH_CW=0

make -s OUT=../lib/libslam2d_noaf.so EXTRA=-DS2D_APPLY_FAST=0
make -s OUT=../lib/libslam2d_nt.so EXTRA=-DS2D_NT_STORE=1
make -s OUT=../lib/libslam2d_oct.so EXTRA=-DS2D_OCTET=1
make -s OUT=../lib/libslam2d_oct2.so EXTRA="-DS2D_OCTET=2 -DS2D_UPD_MINB=6"
make -s OUT=../lib/libslam2d_wedge.so EXTRA=-DS2D_WEDGE=1
make -s OUT=../lib/libslam2d_batch.so EXTRA=-DS2D_CULL_BATCH=1
make -s OUT=../lib/libslam2d_batchw.so EXTRA="-DS2D_CULL_BATCH=1 -DS2D_WEDGE=1"
