# Hector parity tests with the product library, then a same-box A/B of library variants:
#   tools/gpu_test_ab.sh <tag> <variant>...   (see tools/ab_bench.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1; shift; mkdir -p $R/gpurun_out/$T; cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_fullsize_gpu.py tests/test_backend_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo "FAIL pytest"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
BENCH_ARGS="${BENCH_ARGS:---steps 20 --warmup 5}" timeout -k 10 600 bash tools/ab_bench.sh $T "$@"
