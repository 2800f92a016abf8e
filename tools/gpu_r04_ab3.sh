#!/bin/bash
# Round-4 GPU session 3: parity suite (clip update kernel + apply fast path + chain-wave match = default), same-box
# A/B of the apply fast path (noaf) and of the match variants (r3m: round 3's chain, cw1: one term buffer) at 2048
# and 2560 streams, the driver's exact command, rocprofv3 profile with the instruction pass.
#   tools/gpu_r04_ab3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04d}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "FAIL pytest"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 900 bash tools/ab_bench.sh $T main noaf r3m cw1 || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --streams 2560" timeout -k 10 600 bash tools/ab_bench.sh ${T}_2560 main cw1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'),'frac',r.get('frac'),'pose',d['pose_vs_ref']['exact_frac_vs_reference_order'])"
bash tools/profile_gpu.sh $T --steps 20 --warmup 5 > $O/profile.log 2>&1 || { echo "FAIL profile"; tail -20 $O/profile.log; exit 1; }
echo profile ok
