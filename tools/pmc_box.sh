#!/bin/bash
# Per-box memory-system counters of the Hector kernels (one rocprofv3 --pmc pass per counter group, as the
# MI355X guide prescribes): address translation (TCP UTCL1 + GRBM UTCL2 busy), DRAM request credit stalls and
# SQ wave / wait cycles.  Compare two leases to attribute a box-to-box gap that the shader clock does not explain.
#   tools/pmc_box.sh <tag> [bench args...]
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/pmcbox_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_LEVEL_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/bench.py" \
      --no-cpu-baseline --no-copy-probe --no-timing --steps 5 --warmup 2 "$@" > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import csv, glob, sys, collections
agg = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("s2d::", "").replace("void ", "")
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for (k, c), v in sorted(agg.items()):
    if k.startswith(("hs_update", "hs_match")):
        print(f"{k:30s} {c:40s} {v / max(cnt[(k, c)], 1):18.0f}")
PY
