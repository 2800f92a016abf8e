# Karto: parity, then same-box A/B vs the HEAD build (sequential batch and loop window)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-kt}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_karto_gpu.py tests/test_fullsize_gpu.py -k "karto or Karto or kt" > gpurun_out/${TAG}_test.log 2>&1 &&
BENCH_ARGS="--config karto" timeout -k 10 600 tools/ab_bench.sh ${TAG} main prev > gpurun_out/${TAG}_ab.log 2>&1 &&
BENCH_ARGS="--config karto_loop" timeout -k 10 600 tools/ab_bench.sh ${TAG}l main prev > gpurun_out/${TAG}l_ab.log 2>&1
