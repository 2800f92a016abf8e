#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of library variants over bench.py (separate passes):  tools/pmc_fetch_ab.sh <tag> <variant>...
#   then: python3 tools/pmc_cmp.py hs_update gpurun_out/pmcf_<tag>_<v>...
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_$v.so; fi
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  OUT=$ROOT/gpurun_out/pmcf_${TAG}_$v; mkdir -p "$OUT"
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    SLAM2D_LIB=$lib timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe --steps 5 --warmup 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  done
done
