# late round-2 refresh: PL-ICP and Karto bench lines (CPU baselines included) and their profiles
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02n; cd $R
for c in "plicp:--config plicp" "karto:--config karto" "karto_loop:--config karto_loop"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 400 python3 bench.py $args > gpurun_out/r02n/$name.json 2> gpurun_out/r02n/$name.err || { echo "FAIL $name"; exit 1; }
  echo "done $name"
done
tools/profile_gpu.sh r02q --config plicp > gpurun_out/r02q.log 2>&1 &&
tools/profile_gpu.sh r02t --config karto > gpurun_out/r02t.log 2>&1
