# PL-ICP: parity, then same-box A/B vs the HEAD build
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-pl}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_plicp_gpu.py tests/test_backend_gpu.py > gpurun_out/${TAG}_test.log 2>&1 &&
BENCH_ARGS="--config plicp" timeout -k 10 600 tools/ab_bench.sh ${TAG} main prev > gpurun_out/${TAG}_ab.log 2>&1
