#!/bin/bash
# Ring-ordered cursor update kernel vs the round-3 clipping kernel (SLAM2D_UPD_KERNEL=clip) on one box:
# Hector parity tests (default = ring), bench A/B (two alternations), PMC instruction counts of both.
#   tools/gpu_ring_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-ring}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_fullsize_gpu.py tests/test_backend_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "FAIL pytest"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 600 bash tools/ab_bench.sh $T main main+SLAM2D_UPD_KERNEL=clip || exit 1
KPREFIX=hs_update timeout -k 10 500 bash tools/pmc_ab.sh $T main main+SLAM2D_UPD_KERNEL=clip > $O/pmc_ring.txt 2>&1 || { echo "FAIL pmc"; tail $O/pmc_ring.txt; exit 1; }
cat $O/pmc_ring.txt
