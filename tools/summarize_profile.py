#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh run into profiles/ (committed evidence).

  python tools/summarize_profile.py <tag> [round]      e.g.  r01s r01

Reads gpurun_out/prof_<tag>/{trace,pmc_fetch,pmc_write}/ and the bench line of the traced run, and
writes
  profiles/<round>/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<round>/<tag>_summary.md         per-kernel avg duration, FETCH_SIZE, WRITE_SIZE, bytes
  profiles/pmc_traffic.json                 per (kernel, config, streams) HBM bytes per launch,
                                            read by bench.py for roofline.traffic
FETCH_SIZE / WRITE_SIZE are in KB.  gfx950 FETCH_SIZE tallies 128-B read requests at 64 B
(MI355X_MICROARCH.md, HBM/rocprofv3 section), so traffic = 2 x FETCH_SIZE + WRITE_SIZE.
"""
import collections
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


INSTS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVES")


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "").replace("s2d::", "")


def main():
    tag = sys.argv[1]
    rnd = sys.argv[2] if len(sys.argv) > 2 else tag[:3]
    src = os.path.join(REPO, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    with open(os.path.join(src, "bench_trace.json")) as f:
        bench = json.loads([ln for ln in f if ln.startswith("{")][-1])
    cfg = bench["config"]["config"]
    streams = next((bench["config"][k] for k in ("streams_per_gpu", "matches_per_gpu", "pairs_per_gpu", "particles_per_gpu")
                    if k in bench["config"]), None)
    # the workload key bench.py matches on (Hector lines carry semantics and summation order)
    wkey = {"config": cfg, "streams": streams}
    for k, field in (("semantics", "semantics"), ("order", "reduction_order"), ("kernel_src", "kernel_src"),
                     ("issue_split", "issue_split")):
        if field in bench["config"]:
            wkey[k] = bench["config"][field]

    dur = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]))
    pmc = collections.defaultdict(dict)
    # the instruction pass (SQ_INSTS_*, SQ_*_CYCLES) is optional: summaries of earlier rounds have none
    passes = [("pmc_fetch", ("FETCH_SIZE",)), ("pmc_write", ("WRITE_SIZE",)), ("pmc_insts", INSTS)]
    for sub, ctrs in passes:
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path) and sub == "pmc_insts":
            continue
        acc = collections.defaultdict(list)
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] in ctrs:
                    acc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, ctr), v in acc.items():
            pmc[k][ctr] = sum(v) / len(v)

    lines = [f"# rocprofv3 summary `{tag}` ({cfg}, {streams} units/GPU)", "",
             f"bench line of the traced run: value {bench['value']} {bench['unit']}, ms/step {bench['ms_per_step']}", "",
             "| kernel | calls | avg us | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch (2F+W) | GB/s "
             "| VALU insts | SALU insts | LDS insts | wave cycles |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    entries = []
    for k, (calls, avg) in sorted(dur.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        fe, wr = pmc.get(k, {}).get("FETCH_SIZE"), pmc.get(k, {}).get("WRITE_SIZE")
        tb = int((2 * fe + wr) * 1024) if fe is not None and wr is not None else None
        gbs = f"{tb / avg:.1f}" if tb else "-"
        ins = {c: pmc.get(k, {}).get(c) for c in INSTS}
        fmt = lambda v: f"{v:.0f}" if v is not None else "-"  # noqa: E731
        lines.append(f"| {k} | {calls} | {avg / 1e3:.1f} | {fe if fe is not None else '-'} | "
                     f"{wr if wr is not None else '-'} | {tb if tb else '-'} | {gbs} | {fmt(ins['SQ_INSTS_VALU'])} | "
                     f"{fmt(ins['SQ_INSTS_SALU'])} | {fmt(ins['SQ_INSTS_LDS'])} | {fmt(ins['SQ_WAVE_CYCLES'])} |")
        if tb and k.startswith(("hs_", "kt_", "gm_", "pl_")):
            e = {"kernel": k, **wkey, "avg_ns": avg,
                 "fetch_kb": fe, "write_kb": wr, "traffic_bytes_per_launch": tb,
                 "source": f"profiles/{rnd}/{tag}_summary.md"}
            if ins["SQ_INSTS_VALU"] is not None:
                e.update({"insts_valu": ins["SQ_INSTS_VALU"], "insts_salu": ins["SQ_INSTS_SALU"],
                          "insts_lds": ins["SQ_INSTS_LDS"], "wave_cycles": ins["SQ_WAVE_CYCLES"],
                          "busy_cycles": ins["SQ_BUSY_CYCLES"], "waves": ins["SQ_WAVES"]})
            entries.append(e)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")

    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {"entries": []}
    def ident(e):
        return (e["kernel"], e["config"], e["streams"], e.get("semantics"), e.get("order"), e.get("kernel_src"),
                e.get("issue_split"))
    keep = [e for e in d["entries"] if ident(e) not in {ident(n) for n in entries}]
    d["entries"] = keep + entries
    with open(path, "w") as f:
        json.dump(d, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
