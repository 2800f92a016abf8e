cd $GRAFT_REPO_ROOT && BENCH_ARGS="--steps 10 --warmup 3" bash tools/ab_bench.sh seq1 h0 main main+SLAM2D_PIPELINE=1 main+SLAM2D_MATCH_ORDER=tree
