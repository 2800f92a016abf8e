#!/bin/bash
# A/B the library variants in lib/ in ONE GPU session: tools/ab_bench.sh <tag> <variant>... (variant "main" = libslam2d.so)
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$ROOT/gpurun_out"
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_$v.so; fi
    SLAM2D_LIB=$lib timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline $BENCH_ARGS > "$ROOT/gpurun_out/ab_${TAG}_${v}_$round.json" 2>/dev/null || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], round(d['value']), r['kernel_ms_per_step'], r['frac'])" "$ROOT/gpurun_out/ab_${TAG}_${v}_$round.json" "$v"
  done
done
