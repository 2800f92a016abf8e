# round-2 measurement set: every bench config once (CPU baselines included), then the north-star profile
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/r02m; cd $R
for c in "northstar:" "reference:--semantics reference" "c2:--config c2" "c3:--config c3" "gmapping:--config gmapping" \
         "plicp:--config plicp" "karto:--config karto" "karto_loop:--config karto_loop"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 400 python3 bench.py $args > gpurun_out/r02m/$name.json 2> gpurun_out/r02m/$name.err || { echo "FAIL $name"; exit 1; }
  echo "done $name"
done
tools/profile_gpu.sh r02z > gpurun_out/r02z.log 2>&1
