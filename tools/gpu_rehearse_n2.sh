# N > 1 bench path rehearsed on ONE GPU: 2 ranks (gloo timing collectives) of the default Hector bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/n2; mkdir -p $O; cd $R
BENCH_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --streams 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "rc $?"; tail -3 $O/bench.err; cat $O/bench.json | cut -c1-600
