# round 3 profiles: north star (forced map update) and the node's gate, reference summation order
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile_gpu.sh r03q --steps 10 --warmup 3 > gpurun_out/r03q.log 2>&1 || { echo "FAIL r03q"; tail -5 gpurun_out/r03q.log; exit 1; }
echo "r03q ok"
bash tools/profile_gpu.sh r03r --steps 10 --warmup 3 --semantics reference > gpurun_out/r03r.log 2>&1 || { echo "FAIL r03r"; tail -5 gpurun_out/r03r.log; exit 1; }
echo "r03r ok"
