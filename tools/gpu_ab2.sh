# Hector parity, then same-box A/B main vs prev (HEAD build) in forced-update and reference-gate modes
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
TAG=${1:-ab}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_backend_gpu.py > gpurun_out/${TAG}_test.log 2>&1 &&
timeout -k 10 600 tools/ab_bench.sh $TAG main prev > gpurun_out/${TAG}_ab.log 2>&1 &&
BENCH_ARGS="--semantics reference" timeout -k 10 600 tools/ab_bench.sh ${TAG}r main prev > gpurun_out/${TAG}r_ab.log 2>&1
