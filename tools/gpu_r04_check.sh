#!/bin/bash
# Round-4 last check on a fresh box: smoke() and the GPU parity suite on the committed tree.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out/r04l
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04l/smoke.log 2>&1 || { echo FAIL smoke; tail -20 gpurun_out/r04l/smoke.log; exit 1; }
tail -2 gpurun_out/r04l/smoke.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04l/pytest.log 2>&1 || { echo FAIL pytest; tail -20 gpurun_out/r04l/pytest.log; exit 1; }
tail -1 gpurun_out/r04l/pytest.log
