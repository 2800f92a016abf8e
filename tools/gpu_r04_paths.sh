#!/bin/bash
# Round-4 refresh of the other paths' bench lines on the final kernels (one lease): the node gate (reference
# map-update semantics), c2, c3, GMapping, PL-ICP, Karto (batch and loop window).
#   tools/gpu_r04_paths.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}; T=${1:-r04m}; O=$R/gpurun_out/$T; mkdir -p $O; cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['metric'][:40], round(d['value']), d['unit'], d['ms_per_step'])" $O/$n.json $n
}
run gate --semantics reference
run c2 --config c2
run c3 --config c3
run gmapping --config gmapping
run plicp --config plicp
run karto --config karto
run karto_loop --config karto_loop
