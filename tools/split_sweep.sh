# north-star update split sweep at the default fleet: SLAM2D_UPD_SPLIT variants, two alternating rounds
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/split_${1:-r02}; mkdir -p $OUT; cd $R
for rnd in 1; do
  for sp in def 3,1,1 4,1,1 2,2,1 3,2,1 4,2,1 6,2,1; do
    if [ $sp = def ]; then unset SLAM2D_UPD_SPLIT; else export SLAM2D_UPD_SPLIT=$sp; fi
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-copy-probe > $OUT/s${sp}_$rnd.json 2> $OUT/s${sp}_$rnd.err || { echo "FAIL $sp"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], r['kernel_ms_per_step'])" $OUT/s${sp}_$rnd.json $sp
  done
done
