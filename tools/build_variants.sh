#!/bin/bash
# Compile-time A/B variants of the product library (same sources, other -D switches) next to libslam2d.so:
#   th64  ring update kernel with 64-row tiles and 512-thread workgroups (S2D_RING_TH=64)
#   cw1   chain-wave match with one term buffer (S2D_CW_BUFS=1: 31 KB of LDS, 5 workgroups per CU)
#   r3m   round 3's match chain (S2D_MATCH_CW=0)
#   noaf  no apply fast path (S2D_APPLY_FAST=0)
set -e
cd "$(dirname "$0")/../creating-2d-laser-slam-from-scratch_amd/csrc"
make -s
make -s OUT=../lib/libslam2d_th64.so EXTRA=-DS2D_RING_TH=64
make -s OUT=../lib/libslam2d_cw1.so EXTRA=-DS2D_CW_BUFS=1
make -s OUT=../lib/libslam2d_r3m.so EXTRA=-DS2D_MATCH_CW=0
make -s OUT=../lib/libslam2d_th64cw1.so "EXTRA=-DS2D_RING_TH=64 -DS2D_CW_BUFS=1"
make -s OUT=../lib/libslam2d_noaf.so EXTRA=-DS2D_APPLY_FAST=0
