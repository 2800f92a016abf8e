#!/bin/bash
# A/B of the current build against lib/libslam2d_head.so: hector parity, bench A/B, then SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-x}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hector_gpu.py tests/test_ingest_gpu.py > gpurun_out/${T}_pytest.log 2>&1 && tail -2 gpurun_out/${T}_pytest.log &&
BENCH_ARGS="--steps 10 --warmup 3" bash tools/ab_bench.sh $T ${AB:-head main} &&
bash tools/pmc_ab.sh $T main
