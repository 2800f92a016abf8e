#!/bin/bash
# Round-4 GPU session: the update's workgroup split per level at the 3840-stream fleet (environment only, same
# library): the default (level 0 in 2 parts), 3 / 4 parts at level 0, and one workgroup per level.
#   tools/gpu_r04_split.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04t}; cd $R
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 900 bash tools/ab_bench.sh ${T} main main+SLAM2D_UPD_SPLIT=3,1,1 \
    main+SLAM2D_UPD_SPLIT=4,2,1 main+SLAM2D_UPD_PARTS=1,1,1 || exit 1
