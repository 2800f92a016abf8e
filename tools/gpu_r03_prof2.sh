# round 3 profiles after the raster / culling work: north star (forced map update) and the node's gate
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_gpu.sh r03u --steps 10 --warmup 3 > gpurun_out/r03u.log 2>&1 || { echo "FAIL r03u"; tail -5 gpurun_out/r03u.log; exit 1; }
echo "r03u ok"
bash tools/profile_gpu.sh r03v --steps 10 --warmup 3 --semantics reference > gpurun_out/r03v.log 2>&1 || { echo "FAIL r03v"; tail -5 gpurun_out/r03v.log; exit 1; }
echo "r03v ok"
