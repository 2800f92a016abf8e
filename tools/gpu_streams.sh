#!/bin/bash
# update-kernel time vs fleet size (throughput vs latency): tools/gpu_streams.sh <tag> [streams...]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=$1; shift
for B in "$@"; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-copy-probe --steps 10 --warmup 3 --streams $B > gpurun_out/st_${T}_$B.json 2>/dev/null || { echo "FAIL $B"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], round(d['value']), r['kernel_ms_per_step'])" gpurun_out/st_${T}_$B.json $B
done
