#!/bin/bash
# Round-4 closing session 2 (after the mark-read packing): the driver's exact bench command, rocprofv3 trace +
# counter passes at the default north-star fleet (3840 streams), then a 5120-stream fleet for comparison.
#   tools/gpu_r04_final2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04k}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'))"
bash tools/profile_gpu.sh $T --steps 20 --warmup 5 > $O/profile.log 2>&1 || { echo "FAIL profile"; tail -20 $O/profile.log; exit 1; }
echo profile ok
BENCH_ARGS="--steps 20 --warmup 5 --streams 5120" timeout -k 10 500 bash tools/ab_bench.sh ${T}_5120 main || exit 1
