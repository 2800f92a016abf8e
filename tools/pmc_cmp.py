#!/usr/bin/env python3
"""Side-by-side PMC counters of tools/pmc_ab.sh runs: python tools/pmc_cmp.py <kernel-prefix> gpurun_out/pmcab_<tag>_<v>..."""
import collections
import csv
import glob
import sys

pre, dirs = sys.argv[1], sys.argv[2:]
tab = {}
for d in dirs:
    agg = collections.defaultdict(float); cnt = collections.Counter()
    for f in glob.glob(d + "/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("s2d::", "").replace("void ", "")
            if k.startswith(pre):
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[r["Counter_Name"]] += 1
    tab[d] = {c: agg[c] / cnt[c] for c in agg}
names = sorted(set(c for t in tab.values() for c in t))
print(f"{'counter':24s}" + "".join(f"{d.split('pmcab_')[-1][:22]:>24s}" for d in dirs))
for c in names:
    print(f"{c:24s}" + "".join(f"{tab[d].get(c, 0):24.0f}" for d in dirs))
