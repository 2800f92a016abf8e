#!/bin/bash
# A/B library variants in ONE GPU session:  tools/ab_bench.sh <tag> <variant>...
#   variant = name[+KEY=VAL]  -> lib/ab/libslam2d_<name>.so ("main" = libslam2d.so), optional env KEY=VAL
#             (+ARGS=a/b: extra bench.py arguments for this variant instead, e.g. main+ARGS=--streams/5120)
# BENCH_ARGS (env) is appended to every bench.py call; AB_ROUNDS (env, default 2) rounds.
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$ROOT/gpurun_out"
# rounds alternate the order (A B, B A, ...): a lease's clock drifts over a session (the second library of a
# pair ran 20-40 MHz lower in round 5's A/Bs), so a fixed order biases against the later variants
SPECS=("$@")
for round in $(seq 1 "${AB_ROUNDS:-2}"); do
  ORDER=("${SPECS[@]}")
  if [ $((round % 2)) -eq 0 ]; then ORDER=(); for ((k=${#SPECS[@]}-1; k>=0; k--)); do ORDER+=("${SPECS[$k]}"); done; fi
  for spec in "${ORDER[@]}"; do
    v=${spec%%+*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*+}
    # +ARGS=a/b/c: extra bench.py arguments of this variant (slashes become spaces), not an environment variable
    vargs=""; case "$envs" in ARGS=*) vargs=${envs#ARGS=}; vargs=${vargs//\// }; envs="" ;; esac
    if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_$v.so; fi
    tagv=$(echo "$spec" | tr '+=/' '___')
    env SLAM2D_LIB=$lib $envs timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe $BENCH_ARGS $vargs > "$ROOT/gpurun_out/ab_${TAG}_${tagv}_$round.json" 2>/dev/null || { echo "FAIL $spec"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));r=d.get('roofline') or {};print(sys.argv[2], round(d['value']), r.get('kernel_ms_per_step'), 'sclk', r.get('update_sclk_mhz'), r.get('match_sclk_mhz'), r.get('frac'), d['config'].get('kernel_ms', ''))" "$ROOT/gpurun_out/ab_${TAG}_${tagv}_$round.json" "$spec"
  done
done
