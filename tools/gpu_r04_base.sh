#!/bin/bash
# Round-4 baseline on a fresh box: GPU parity suite, the driver's exact bench command (with the shader-clock
# probe), the self-launched 2-rank rehearsal (gloo timing collectives, one GPU), and a rocprofv3 profile
# with the instruction-count pass.  usage: tools/gpu_r04_base.sh <tag> [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04a}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "FAIL pytest"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.json 2> $O/driver_cmd.err \
  || { echo "FAIL bench"; tail -20 $O/driver_cmd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/driver_cmd.json'));r=d['roofline'];print('value',d['value'],'ms',d['ms_per_step'],'kms',r['kernel_ms_per_step'],'sclk',r.get('update_sclk_mhz'),r.get('match_sclk_mhz'))"
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
