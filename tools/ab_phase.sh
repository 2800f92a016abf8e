cd $GRAFT_REPO_ROOT && BENCH_ARGS="--steps 10 --warmup 3" bash tools/ab_bench.sh phase main phase1 phase2
