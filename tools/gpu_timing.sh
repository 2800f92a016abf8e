# does per-kernel event timing inside the timed region cost wall time?  (same box, alternating)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-copy-probe > gpurun_out/tm_on_$r.json 2>/dev/null &&
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-copy-probe --no-timing > gpurun_out/tm_off_$r.json 2>/dev/null || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/tm_on_$r.json'));b=json.load(open('gpurun_out/tm_off_$r.json'));print('on',a['ms_per_step'],'off',b['ms_per_step'])"
done
