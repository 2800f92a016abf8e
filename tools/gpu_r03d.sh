set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03d; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hector_gpu.py tests/test_ingest_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { echo "FAIL tests"; tail -30 $O/pytest.log; exit 1; }
echo "tests ok: $(tail -1 $O/pytest.log)"
BENCH_ARGS="--steps 10 --warmup 3" bash tools/ab_bench.sh mul24 h4 main
