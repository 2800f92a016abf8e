#!/bin/bash
# streams-per-GPU sweep of the north-star bench (B = 1 ... 4096), one bench.py line each.
# usage: tools/sweep_streams.sh <tag> [extra bench args]
TAG=${1:-sweep}; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/sweep_$TAG; mkdir -p "$OUT"
for B in 1 4 16 64 256 1024 2048 4096; do
  timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe --steps 10 --warmup 3 --streams $B "$@" \
      > "$OUT/b$B.json" 2> "$OUT/b$B.err" || { echo "B=$B failed"; tail -3 "$OUT/b$B.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'] or {};print(sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_step'), r.get('frac'))" "$OUT/b$B.json" $B
done
