#!/bin/bash
# Round-4 GPU session 2: parity suite (ring update kernel + chain-wave match = default), the driver's exact
# bench command, same-box A/B of update kernel (ring / clip) and match variants (two buffers / one buffer /
# round-3 chain), 2-rank self-launched rehearsal, rocprofv3 profile with the instruction pass.
#   tools/gpu_r04_ab2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04c}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
PRC=$?
tail -3 $O/pytest.log
if [ $PRC -ne 0 ]; then
  echo "FAIL pytest rc=$PRC"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20
  # the round-3 kernels alone, so the session still yields the baseline line
  SLAM2D_LIB=$R/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_r3m.so SLAM2D_UPD_KERNEL=clip timeout -k 10 300 \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd_r3.json 2> $O/driver_cmd_r3.err
  exit 1
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'),'pose',d['pose_vs_ref']['exact_frac_vs_reference_order'])"
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 900 bash tools/ab_bench.sh $T main main+SLAM2D_UPD_KERNEL=clip th64 cw1 || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --streams 2560" timeout -k 10 600 bash tools/ab_bench.sh ${T}_2560 cw1 th64cw1 || exit 1
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --streams 512 --no-cpu-baseline --steps 10 \
  > $O/n2_northstar.json 2> $O/n2_northstar.err || { echo "FAIL n2 northstar"; tail -20 $O/n2_northstar.err; exit 1; }
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --config gmapping --weights torch --no-cpu-baseline \
  > $O/n2_gmapping.json 2> $O/n2_gmapping.err || { echo "FAIL n2 gmapping"; tail -20 $O/n2_gmapping.err; exit 1; }
python3 -c "
import json
for f in ('n2_northstar', 'n2_gmapping'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['n_gpus'], d['value'], d['config'].get('global_batch'), d['config'].get('particles'))"
bash tools/profile_gpu.sh $T --steps 20 --warmup 5 > $O/profile.log 2>&1 || { echo "FAIL profile"; tail -20 $O/profile.log; exit 1; }
echo profile ok
