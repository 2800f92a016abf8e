# 4x4-blocked tiles: Hector parity tests, then same-box A/B against HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03c; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_backend_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "FAIL tests"; tail -30 $O/pytest.log; exit 1; }
echo "tests ok"; tail -1 $O/pytest.log
BENCH_ARGS="--steps 10 --warmup 3" bash tools/ab_bench.sh blk h3 main
