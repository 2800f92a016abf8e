# update kernel rays in registers: Hector parity (both instances), then same-box A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/rreg
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_fullsize_gpu.py > gpurun_out/rreg/test.log 2>&1 || { echo "FAIL test"; tail -30 gpurun_out/rreg/test.log; exit 1; }
tail -2 gpurun_out/rreg/test.log
SLAM2D_UPD_RAYS_LDS=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py > gpurun_out/rreg/test_lds.log 2>&1 || { echo "FAIL test_lds"; tail -30 gpurun_out/rreg/test_lds.log; exit 1; }
tail -2 gpurun_out/rreg/test_lds.log
timeout -k 10 600 tools/ab_bench.sh rreg main main+SLAM2D_UPD_RAYS_LDS=1
BENCH_ARGS="--streams 1024" timeout -k 10 600 tools/ab_bench.sh rreg1k main main+SLAM2D_UPD_RAYS_LDS=1
