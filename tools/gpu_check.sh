# full GPU check: parity tests, smoke, default (north-star) bench; results under gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT; T=${1:-check}; mkdir -p $R/gpurun_out/$T; cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { echo "FAIL pytest"; tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.log 2>&1 || { echo "FAIL smoke"; tail -20 gpurun_out/$T/smoke.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/$T/northstar.json 2> gpurun_out/$T/northstar.err || { echo "FAIL bench"; tail -20 gpurun_out/$T/northstar.err; exit 1; }
cat gpurun_out/$T/northstar.json
