# GMapping borrow-select walk: parity, then same-box A/B vs the HEAD build
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gmapping_gpu.py tests/test_hector_gpu.py > gpurun_out/gmw_test.log 2>&1 &&
BENCH_ARGS="--config gmapping" timeout -k 10 600 tools/ab_bench.sh gmw main prev > gpurun_out/gmw_ab.log 2>&1 &&
timeout -k 10 600 tools/ab_bench.sh hwexp main hwexp > gpurun_out/hwexp_ab.log 2>&1
