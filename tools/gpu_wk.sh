# default K/W vs longer warmup / timed region, fresh box, alternating
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/wk_def_$r.json 2>gpurun_out/wk_def_$r.err &&
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --warmup 30 --steps 100 > gpurun_out/wk_long_$r.json 2>gpurun_out/wk_long_$r.err || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/wk_def_$r.json'));b=json.load(open('gpurun_out/wk_long_$r.json'));print('def',a['value'],a['ms_per_step'],'long',b['value'],b['ms_per_step'])"
done
grep -h "generated" gpurun_out/wk_*_1.err
