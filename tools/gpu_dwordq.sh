# dwordq pricing: parity with the variant library, same-box A/B, FETCH/WRITE of both
set -o pipefail
R=$GRAFT_REPO_ROOT; T=dwq; mkdir -p $R/gpurun_out/$T; cd $R
SLAM2D_LIB=$R/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_dwordq.so timeout -k 10 300 python3 -u -m pytest tests/test_hector_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo "FAIL pytest"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 400 bash tools/ab_bench.sh $T main dwordq || exit 1
timeout -k 10 400 bash tools/pmc_fetch_ab.sh $T main dwordq
