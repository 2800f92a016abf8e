#!/bin/bash
# Round-4 GPU session 11: the match prologue and every level start at priority 2 as well
# (S2D_PROLOGUE_PRIO=1, new default) -- parity suite, A/B against default-priority prologue (pp0) at the north-star fleet,
# then the driver's command and the closing profile of these kernels.
#   tools/gpu_r04_ab11.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04s}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "FAIL pytest"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 600 bash tools/ab_bench.sh ${T} main pp0 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'))"
bash tools/profile_gpu.sh $T --steps 20 --warmup 5 > $O/profile.log 2>&1 || { echo "FAIL profile"; tail -20 $O/profile.log; exit 1; }
echo profile ok
