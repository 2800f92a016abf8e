# round-2 side-path profiles: PL-ICP, GMapping, Karto (scan and loop windows)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
tools/profile_gpu.sh r02p --config plicp > gpurun_out/r02p.log 2>&1 &&
tools/profile_gpu.sh r02g --config gmapping > gpurun_out/r02g.log 2>&1 &&
tools/profile_gpu.sh r02k --config karto_loop > gpurun_out/r02k.log 2>&1 &&
tools/profile_gpu.sh r02s --config karto > gpurun_out/r02s.log 2>&1
