#!/bin/bash
# Round-4 GPU session 7: the update's mark read packed by byte permutes (S2D_PACK_PERM=1, the new default) --
# the parity suite on it, then the A/B against the compact-nibble packing (pk0) at the north-star fleet.
#   tools/gpu_r04_ab7.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04j}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { echo "FAIL pytest"; grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--steps 20 --warmup 5" timeout -k 10 900 bash tools/ab_bench.sh ${T} main pk0 || exit 1
timeout -k 10 300 bash tools/pmc_ab.sh ${T} main pk0 > $O/pmc_ab.txt 2>&1 || { echo "FAIL pmc_ab"; tail $O/pmc_ab.txt; exit 1; }
grep -E "INSTS_VALU|WAVE_CYCLES|WAIT_INST_ANY" $O/pmc_ab.txt
