#!/bin/bash
# Round-4 GPU session 5: the parity suite, then cone-culled fan groups (S2D_WEDGE) and whole-sector apply stores
# (S2D_OCTET 1 / 2) -- each variant's parity on the bit-exact Hector tests, the A/B at the north-star fleet against
# the default, the non-temporal stores and a per-stream pad -- the driver's exact command and the per-box
# memory-system counters.
#   tools/gpu_r04_ab5.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04f}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
L=$R/creating-2d-laser-slam-from-scratch_amd/lib
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "FAIL pytest"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
K="bitexact or dense or golden or long_rays or hand_built or clamp or batch_sizes or degenerate or ragged"
for v in wedge oct oct2; do
  SLAM2D_LIB=$L/libslam2d_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_hector_gpu.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1 \
    || { echo "FAIL pytest $v"; grep -E "FAILED|Error|assert" $O/pytest_$v.log | head -20; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
BENCH_ARGS="--steps 20 --warmup 5 --streams 2560" timeout -k 10 900 bash tools/ab_bench.sh ${T} main wedge oct oct2 nt \
    main+SLAM2D_STREAM_PAD=4352 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'),'copy',r.get('attainable_copy_GBps'),'pose',d['pose_vs_ref']['exact_frac_vs_reference_order'])"
timeout -k 10 400 bash tools/pmc_box.sh $T > $O/pmc_box.log 2>&1 || { echo "FAIL pmc_box"; tail $O/pmc_box.log; exit 1; }
cat gpurun_out/pmcbox_$T/summary.txt
