#!/bin/bash
# Round-4 closing GPU session: tools/gpu_r04_base.sh (parity suite, the driver's exact bench command, the
# self-launched 2-rank rehearsal, rocprofv3 trace + counter passes at the default north-star fleet), then the
# 3840-stream fleet for comparison.   usage: tools/gpu_r04_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04h}; cd $R
bash tools/gpu_r04_base.sh $T || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --streams 3840" timeout -k 10 400 bash tools/ab_bench.sh ${T}_3840 main || exit 1
