# end-of-round-3 profiles of the final kernels: north star (forced map update) and the node's gate
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_gpu.sh r03x --steps 10 --warmup 3 > gpurun_out/r03x.log 2>&1 || { echo "FAIL r03x"; tail -5 gpurun_out/r03x.log; exit 1; }
echo "r03x ok"
bash tools/profile_gpu.sh r03y --steps 10 --warmup 3 --semantics reference > gpurun_out/r03y.log 2>&1 || { echo "FAIL r03y"; tail -5 gpurun_out/r03y.log; exit 1; }
echo "r03y ok"
