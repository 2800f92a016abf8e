# LDS flags as plain LDS arrays (no flat accesses): parity (Hector, GMapping) and A/B vs the previous build
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_gmapping_gpu.py > gpurun_out/flat_test.log 2>&1 &&
timeout -k 10 600 tools/ab_bench.sh flat main prev > gpurun_out/flat_ab.log 2>&1 &&
BENCH_ARGS="--config gmapping" timeout -k 10 600 tools/ab_bench.sh flatgm main prev > gpurun_out/flatgm_ab.log 2>&1
