# final kernels: fleet-size sweep of the north star and one long run (K = 100)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sweep3; mkdir -p $O; cd $R
for B in 1024 2048 3072 4096; do
  timeout -k 10 300 python3 bench.py --streams $B --no-cpu-baseline --no-copy-probe > $O/streams_$B.json 2> $O/streams_$B.err || { echo "FAIL $B"; tail -5 $O/streams_$B.err; exit 1; }
  echo "done $B"
done
timeout -k 10 400 python3 bench.py --steps 100 --warmup 30 --no-cpu-baseline > $O/northstar_k100.json 2> $O/northstar_k100.err || { echo "FAIL long"; exit 1; }
echo "done long"
