#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per launch of one kernel across env settings (one PMC pass each):
#   tools/pmc_write_sweep.sh <tag> <kernel substring> "<bench args>" ENV=VAL [ENV=VAL ...]
TAG=$1; KER=$2; ARGS=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
  for ctr in WRITE_SIZE FETCH_SIZE; do
    OUT=$ROOT/gpurun_out/pmcw_${TAG}_$(echo "$spec" | tr '=,/' '___' | tail -c 60)_$ctr
    env $spec timeout -k 10 120 rocprofv3 --pmc $ctr -d "$OUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe --steps 3 --warmup 1 $ARGS > "$OUT.log" 2>&1 || { echo "FAIL $spec $ctr"; exit 1; }
    python3 - "$OUT" "$KER" "$spec" "$ctr" <<'PY'
import csv, glob, sys
vals = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)
        for r in csv.DictReader(open(f)) if sys.argv[2] in r["Kernel_Name"]]
print(sys.argv[3], sys.argv[4], "KB/launch", round(sum(vals) / max(len(vals), 1), 1), "launches", len(vals))
PY
  done
done
