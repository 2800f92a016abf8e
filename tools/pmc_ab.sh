#!/bin/bash
# PMC A/B of library variants over bench.py: tools/pmc_ab.sh <tag> <variant>...  (variant name -> lib/ab/libslam2d_<name>.so, "main")
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
  v=${spec%%+*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*+}
  if [ "$v" = main ]; then lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d.so; else lib=$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/ab/libslam2d_$v.so; fi
  [ -f "$lib" ] || { echo "missing $lib"; exit 1; }
  tagv=$(echo "$spec" | tr '+=' '__')
  OUT=$ROOT/gpurun_out/pmcab_${TAG}_$tagv; mkdir -p "$OUT"
  i=0
  # PMC_SETS="set;set;..." overrides the default three passes (each set within one pass's block limits)
  IFS=';' read -r -a SETS <<< "${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_ADDR_CONFLICT}"
  for set in "${SETS[@]}"; do
    i=$((i+1))
    env SLAM2D_LIB=$lib $envs timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-copy-probe --steps 5 --warmup 2 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  done
  python3 - "$OUT" "$tagv" <<'PY'
import csv, glob, os, sys, collections
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("s2d::", "").replace("void ", "")
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for (k, c), v in sorted(agg.items()):
    if k.startswith(os.environ.get("KPREFIX", "hs_update")): print(sys.argv[2], f"{k:18s} {c:24s} {v/ max(cnt[(k,c)],1):16.0f}")
PY
done
