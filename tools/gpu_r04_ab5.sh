#!/bin/bash
# Round-4 GPU session 5: cone-culled fan groups (S2D_WEDGE) and whole-sector apply stores (S2D_OCTET 1 / 2) --
# parity of the variants on the bit-exact
# update tests, then the A/B against the default and the non-temporal stores at the north-star fleet.
#   tools/gpu_r04_ab5.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
L=$R/creating-2d-laser-slam-from-scratch_amd/lib
K="bitexact or dense or golden or long_rays or hand_built or clamp or batch_sizes or stream_pad"
for v in wedge oct oct2; do
  SLAM2D_LIB=$L/libslam2d_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_hector_gpu.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1 \
    || { echo "FAIL pytest $v"; grep -E "FAILED|Error|assert" $O/pytest_$v.log | head -20; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
BENCH_ARGS="--steps 20 --warmup 5 --streams 2560" timeout -k 10 900 bash tools/ab_bench.sh ${T} main wedge oct oct2 || exit 1
