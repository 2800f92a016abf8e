#!/bin/bash
# Profile bench.py on the GPU box: kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE),
# as MI355X_MICROARCH.md's rocprofv3 section prescribes (one TCC counter group per pass).
# usage: tools/profile_gpu.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS --no-timing > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS --no-timing > "$OUT/bench_write.json" 2> "$OUT/bench_write.err" || exit $?
# instruction counts and cycles (SQ block: <= 8 counters in one pass), for cycle-based comparisons across boxes
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES \
    -d "$OUT/pmc_insts" -o run --output-format csv -- \
    python3 "$ROOT/bench.py" $ARGS --no-timing > "$OUT/bench_insts.json" 2> "$OUT/bench_insts.err" || exit $?
find "$OUT" -name "*.csv" | head -50
