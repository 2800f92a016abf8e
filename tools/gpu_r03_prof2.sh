# round 3 profiles after the raster / culling work: north star (forced map update) and the node's gate
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_gpu.sh r03s --steps 10 --warmup 3 > gpurun_out/r03s.log 2>&1 || { echo "FAIL r03s"; tail -5 gpurun_out/r03s.log; exit 1; }
echo "r03s ok"
bash tools/profile_gpu.sh r03t --steps 10 --warmup 3 --semantics reference > gpurun_out/r03t.log 2>&1 || { echo "FAIL r03t"; tail -5 gpurun_out/r03t.log; exit 1; }
echo "r03t ok"
