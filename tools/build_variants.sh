#!/bin/bash
# Compile-time A/B variants of the product library (same sources, other -D switches) under lib/ab/ (the driver ships only lib/libslam2d.so; lib/ab/ is gpurun-ignored at round end):
#   th64  ring update kernel (opt-in, SLAM2D_UPD_KERNEL=ring) with 64-row tiles and 512-thread workgroups
#   cw2   chain-wave match with two term buffers (S2D_CW_BUFS=2: 38 KB of LDS, 4 workgroups per CU)
#   r3m   round 3's match chain (S2D_MATCH_CW=0)
#   noaf  no apply fast path (S2D_APPLY_FAST=0)
#   nt    non-temporal stores in the update apply (S2D_NT_STORE=1)
#   pk0   round-3 compact-nibble packing of the update's mark bits (S2D_PACK_PERM=0)
#   ing0  ingest chunk loop for every scan (S2D_ING_PRELOAD=0)
#   sc0   per-wave miss conversion in the chain-wave match (S2D_CW_SHARECONV=0)
#   pr0   no raised priority for the match's pre-chain phase (S2D_PRECHAIN_PRIO=0)
#   uprio update waves prioritised by their share of the tile's fan groups (S2D_UPD_PRIO=1)
#   pp0   the match prologue / level starts at default priority (S2D_PROLOGUE_PRIO=0)
# (round 4's oct / oct2 / wedge / batch / batchw variants were measured slower or equal and removed from the
# sources; their code is profiles/r04/update_variants_octet_wedge_batch.patch, results profiles/r04/ab_r04f.md, ab_r04g.md)
set -e
cd "$(dirname "$0")/../creating-2d-laser-slam-from-scratch_amd/csrc"
make -s
make -s OUT=../lib/ab/libslam2d_th64.so EXTRA=-DS2D_RING_TH=64
make -s OUT=../lib/ab/libslam2d_cw2.so EXTRA=-DS2D_CW_BUFS=2
make -s OUT=../lib/ab/libslam2d_r3m.so EXTRA=-DS2D_MATCH_CW=0

make -s OUT=../lib/ab/libslam2d_noaf.so EXTRA=-DS2D_APPLY_FAST=0
make -s OUT=../lib/ab/libslam2d_nt.so EXTRA=-DS2D_NT_STORE=1
make -s OUT=../lib/ab/libslam2d_pk0.so EXTRA=-DS2D_PACK_PERM=0
make -s OUT=../lib/ab/libslam2d_ing0.so EXTRA=-DS2D_ING_PRELOAD=0
make -s OUT=../lib/ab/libslam2d_sc0.so EXTRA=-DS2D_CW_SHARECONV=0
make -s OUT=../lib/ab/libslam2d_pr0.so EXTRA=-DS2D_PRECHAIN_PRIO=0
make -s OUT=../lib/ab/libslam2d_uprio.so EXTRA=-DS2D_UPD_PRIO=1
make -s OUT=../lib/ab/libslam2d_pp0.so EXTRA=-DS2D_PROLOGUE_PRIO=0
