#!/bin/bash
# Round-4 box-spread sample: on whatever lease this lands, the driver's command (clock probe) plus the
# per-box memory-system and SQ issue counters of the final kernels (tools/pmc_box.sh, tools/pmc_ab.sh main).
#   tools/gpu_r04_boxes.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04o}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'),'traffic',r.get('traffic'),'frac',r.get('frac'))"
timeout -k 10 500 bash tools/pmc_box.sh $T > $O/pmc_box.log 2>&1 || { echo "FAIL pmc_box"; tail $O/pmc_box.log; exit 1; }
timeout -k 10 400 bash tools/pmc_ab.sh ${T} main > $O/pmc_ab.txt 2>&1 || { echo "FAIL pmc_ab"; tail $O/pmc_ab.txt; exit 1; }
grep -E "update" gpurun_out/pmcbox_$T/summary.txt
grep -E "INSTS_VALU|ACTIVE_INST_VALU|WAVE_CYCLES|WAIT_INST_ANY|WAIT_ANY|BUSY_CYCLES" $O/pmc_ab.txt
