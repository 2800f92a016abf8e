#!/bin/bash
# A/B library variants in ONE GPU session:  tools/ab_bench.sh <tag> <variant>...
#   variant = name[+KEY=VAL]  -> lib/ab/libslam2d_<name>.so ("main" = libslam2d.so), optional env KEY=VAL
# BENCH_ARGS (env) is appended to every bench.py call.
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$ROOT/gpurun_out"
for round in 1 2; do
  for spec in "$@"; do
    v=${spec%%+*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*+}
    if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_$v.so; fi
    tagv=$(echo "$spec" | tr '+=' '__')
    env SLAM2D_LIB=$lib $envs timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe $BENCH_ARGS > "$ROOT/gpurun_out/ab_${TAG}_${tagv}_$round.json" 2>/dev/null || { echo "FAIL $spec"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline') or {};print(sys.argv[2], round(d['value']), r.get('kernel_ms_per_step'), 'sclk', r.get('update_sclk_mhz'), r.get('match_sclk_mhz'), r.get('frac'), d['config'].get('kernel_ms', ''))" "$ROOT/gpurun_out/ab_${TAG}_${tagv}_$round.json" "$spec"
  done
done
