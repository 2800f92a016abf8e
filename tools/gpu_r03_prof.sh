# round 3 profiles: north star (forced map update) and the node's gate, reference summation order
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_gpu.sh r03p --steps 10 --warmup 3 > gpurun_out/r03p.log 2>&1 || { echo "FAIL r03p"; tail -5 gpurun_out/r03p.log; exit 1; }
echo "r03p ok"
bash tools/profile_gpu.sh r03g --steps 10 --warmup 3 --semantics reference > gpurun_out/r03g.log 2>&1 || { echo "FAIL r03g"; tail -5 gpurun_out/r03g.log; exit 1; }
echo "r03g ok"
