# update-kernel walk variants: parity on the winner candidates, then same-box A/B of the north-star bench
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
L=$R/creating-2d-laser-slam-from-scratch_amd/lib
SLAM2D_LIB=$L/libslam2d_w2.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py > gpurun_out/walk_test_w2.log 2>&1 &&
SLAM2D_LIB=$L/libslam2d_w1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py > gpurun_out/walk_test_w1.log 2>&1 &&
timeout -k 10 600 tools/ab_bench.sh walk main w1 w2 > gpurun_out/walk_ab.log 2>&1
