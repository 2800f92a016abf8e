# end-of-round set: all GPU tests + smoke + north-star bench, reference-gate bench, rocprofv3 profile
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r02f}; cd $R
bash tools/gpu_check.sh $T || exit 1
timeout -k 10 300 python3 bench.py --semantics reference > gpurun_out/$T/reference.json 2> gpurun_out/$T/reference.err || { echo "FAIL ref"; exit 1; }
tools/profile_gpu.sh $T > gpurun_out/$T/prof.log 2>&1 || { echo "FAIL prof"; exit 1; }
echo ok
