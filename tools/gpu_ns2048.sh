# north star at the 2048-stream default: bench lines (forced + reference gate) and the rocprofv3 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r02w}; mkdir -p $R/gpurun_out/$T; cd $R
timeout -k 10 300 python3 bench.py > gpurun_out/$T/northstar.json 2> gpurun_out/$T/northstar.err || { echo "FAIL ns"; exit 1; }
cat gpurun_out/$T/northstar.json
timeout -k 10 300 python3 bench.py --semantics reference > gpurun_out/$T/reference.json 2> gpurun_out/$T/reference.err || { echo "FAIL ref"; exit 1; }
tools/profile_gpu.sh ${T} > gpurun_out/$T/prof.log 2>&1 || { echo "FAIL prof"; exit 1; }
echo ok
