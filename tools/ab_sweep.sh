#!/bin/bash
# Same-box A/B of library variants over a streams sweep: tools/ab_sweep.sh "<B list>" <variant>...
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
BS=$1; shift
for B in $BS; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_$v.so; fi
    SLAM2D_LIB=$lib timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe --steps 10 --warmup 3 --streams $B $BENCH_ARGS > /tmp/abs.json 2>/dev/null || { echo "FAIL $v B=$B"; exit 1; }
    python3 -c "import json,sys;d=json.load(open('/tmp/abs.json'));r=d.get('roofline') or {};print(sys.argv[1], sys.argv[2], d['value'], d['ms_per_step'], r.get('kernel_ms_per_step'))" $B $v
  done
done
