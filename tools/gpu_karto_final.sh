# Karto bench lines (CPU baselines included) and rocprofv3 profiles of both Karto configs
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-r02u}; mkdir -p $R/gpurun_out/$T; cd $R
for c in karto karto_loop; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/$T/$c.json 2> gpurun_out/$T/$c.err || { echo "FAIL $c"; exit 1; }
  echo "done $c"
done
tools/profile_gpu.sh ${T} --config karto > gpurun_out/$T/prof.log 2>&1 || { echo "FAIL prof karto"; exit 1; }
tools/profile_gpu.sh ${T}l --config karto_loop > gpurun_out/$T/profl.log 2>&1 || { echo "FAIL prof karto_loop"; exit 1; }
echo ok
