#!/bin/bash
# Round-4 GPU session 4: parity suite (one-buffer chain-wave match = default now), per-stream pad A/B at 2560 and
# 2048 streams, larger fleets, per-box memory-system counters, the driver's exact command.
#   tools/gpu_r04_ab4.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04e}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "FAIL pytest"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'),'copy',r.get('attainable_copy_GBps'),'pose',d['pose_vs_ref']['exact_frac_vs_reference_order'])"
BENCH_ARGS="--steps 20 --warmup 5 --streams 2560" timeout -k 10 900 bash tools/ab_bench.sh ${T}_pad main main+SLAM2D_STREAM_PAD=256 main+SLAM2D_STREAM_PAD=4352 main+SLAM2D_STREAM_PAD=69888 nt || exit 1
BENCH_ARGS="--steps 20 --warmup 5 --streams 3840" timeout -k 10 600 bash tools/ab_bench.sh ${T}_3840 main || exit 1
timeout -k 10 500 bash tools/pmc_box.sh $T > $O/pmc_box.log 2>&1 || { echo "FAIL pmc_box"; tail $O/pmc_box.log; exit 1; }
cat gpurun_out/pmcbox_$T/summary.txt
