# round 3: the C++ thread test, then north-star benches in both summation orders (short)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03b; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_backend_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_backend.log 2>&1 || { echo "FAIL backend tests"; tail -30 $O/pytest_backend.log; exit 1; }
echo "backend tests ok"
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/ns_ref.json 2> $O/ns_ref.err || { echo "FAIL bench ref"; tail -20 $O/ns_ref.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --order tree > $O/ns_tree.json 2> $O/ns_tree.err || { echo "FAIL bench tree"; tail -20 $O/ns_tree.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --semantics reference > $O/gate_ref.json 2> $O/gate_ref.err || { echo "FAIL bench gate"; tail -20 $O/gate_ref.err; exit 1; }
echo "bench ok"
