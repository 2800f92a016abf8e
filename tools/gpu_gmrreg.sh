# GMapping compute rays in registers: GMapping parity (both instances), then same-box A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/gmrreg
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gmapping_gpu.py tests/test_fullsize_gpu.py -k "gmapping or Gmapping or gm" > gpurun_out/gmrreg/test.log 2>&1 || { echo "FAIL test"; tail -30 gpurun_out/gmrreg/test.log; exit 1; }
tail -2 gpurun_out/gmrreg/test.log
SLAM2D_GM_RAYS_LDS=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gmapping_gpu.py > gpurun_out/gmrreg/test_lds.log 2>&1 || { echo "FAIL test_lds"; tail -30 gpurun_out/gmrreg/test_lds.log; exit 1; }
tail -2 gpurun_out/gmrreg/test_lds.log
BENCH_ARGS="--config gmapping" timeout -k 10 600 tools/ab_bench.sh gmrreg main main+SLAM2D_GM_RAYS_LDS=1
