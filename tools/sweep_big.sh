# north-star bench at large fleets (B = 1024 ... 4096 streams per GPU), one bench.py line each
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/sweep_${1:-big}; mkdir -p $OUT; cd $R
for B in 1024 2048 3072 4096; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-copy-probe --steps 30 --warmup 5 --streams $B > $OUT/b$B.json 2> $OUT/b$B.err || { echo "B=$B failed"; tail -3 $OUT/b$B.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'] or {};print(sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_step'), r.get('frac'), r.get('survey_8d_read_only_frac'), d['pose_vs_ref']['within_tolerance_frac'])" $OUT/b$B.json $B
done
