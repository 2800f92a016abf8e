# Karto coarse tile shape: parity (default shapes, 16 x 16 forced for the loop window), then A/B of SLAM2D_KT_TW
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/kttw_${1:-r02}; mkdir -p $OUT; cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_karto_gpu.py tests/test_fullsize_gpu.py -k "karto or Karto or kt" > $OUT/test.log 2>&1 || { echo "FAIL test"; tail -20 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
SLAM2D_KT_TW=32 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_karto_gpu.py -k "loop or window" > $OUT/test32.log 2>&1 || { echo "FAIL test32"; tail -20 $OUT/test32.log; exit 1; }
tail -2 $OUT/test32.log
for rnd in 1 2; do
  for tw in 16 32 64; do
    for c in karto_loop karto; do
      [ $c = karto ] && [ $tw = 64 ] && continue
      SLAM2D_KT_TW=$tw timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $OUT/${c}_${tw}_$rnd.json 2> $OUT/${c}_${tw}_$rnd.err || { echo "FAIL $c $tw"; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $OUT/${c}_${tw}_$rnd.json $c $tw
    done
  done
done
