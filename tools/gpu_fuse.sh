# fused ingest + walk: Hector GPU parity, then same-box A/B against the separate ingest kernel
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hector_gpu.py tests/test_ingest_gpu.py tests/test_backend_gpu.py tests/test_fullsize_gpu.py > gpurun_out/fuse_test.log 2>&1 &&
SLAM2D_FUSE_INGEST=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ingest_gpu.py > gpurun_out/fuse_test0.log 2>&1 &&
timeout -k 10 600 tools/ab_bench.sh fuse main main+SLAM2D_FUSE_INGEST=0 > gpurun_out/fuse_ab.log 2>&1
