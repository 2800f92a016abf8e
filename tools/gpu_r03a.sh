# round 3, first GPU pass: the Hector parity tests (reference summation order, stored containers,
# reset), then the rest of the -m gpu suite, then a short north-star bench in both summation orders.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03a; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_hector_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_hector.log 2>&1 || { echo "FAIL hector tests"; tail -30 $O/pytest_hector.log; exit 1; }
echo "hector tests ok"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    --deselect tests/test_hector_gpu.py > $O/pytest_all.log 2>&1 || { echo "FAIL gpu tests"; tail -40 $O/pytest_all.log; exit 1; }
echo "all gpu tests ok"
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/ns_ref.json 2> $O/ns_ref.err || { echo "FAIL bench ref"; tail -20 $O/ns_ref.err; exit 1; }
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --order tree > $O/ns_tree.json 2> $O/ns_tree.err || { echo "FAIL bench tree"; tail -20 $O/ns_tree.err; exit 1; }
echo "bench ok"
