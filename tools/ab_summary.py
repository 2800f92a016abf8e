#!/usr/bin/env python3
"""Summarise a tools/ab_bench.sh run: python tools/ab_summary.py <tag> [out.md]

Reads gpurun_out/ab_<tag>_<variant>_<round>.json and prints, per variant, the bench value, ms/step, the
kernels' ms per launch and the clock probe's effective shader clock of every round, plus the mean."""
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def line(path):
    """one bench line in brief: value, ms/step, kernel ms, clocks, frac, kernel_src"""
    d = json.loads([ln for ln in open(path) if ln.startswith("{")][-1])
    r = d.get("roofline") or {}
    k = r.get("kernel_ms_per_step") or {}
    print(os.path.basename(path), round(d["value"]), d["ms_per_step"], k, "sclk", r.get("update_sclk_mhz"),
          r.get("match_sclk_mhz"), "frac", r.get("frac"), "src", d["config"].get("kernel_src"),
          "poses", (d.get("pose_vs_ref") or {}).get("exact_frac_vs_reference_order"))


def main():
    if sys.argv[1] == "--line":
        line(sys.argv[2])
        return
    tag = sys.argv[1]
    rows = defaultdict(list)
    for p in sorted(glob.glob(os.path.join(REPO, "gpurun_out", f"ab_{tag}_*_*.json"))):
        m = re.match(rf"ab_{re.escape(tag)}_(.+)_(\d+)\.json$", os.path.basename(p))
        if not m:
            continue
        try:
            d = json.loads([ln for ln in open(p) if ln.startswith("{")][-1])
        except (IndexError, ValueError):
            continue
        r = d.get("roofline") or {}
        k = r.get("kernel_ms_per_step") or {}
        rows[m.group(1)].append((int(m.group(2)), d["value"], d["ms_per_step"], k.get("match"), k.get("update"),
                                 r.get("match_sclk_mhz"), r.get("update_sclk_mhz"),
                                 (d.get("pose_vs_ref") or {}).get("exact_frac_vs_reference_order")))
    out = [f"# A/B `{tag}`", "", "| variant | round | scans/s | ms/step | match ms | update ms | match MHz | update MHz | poses exact |",
           "|---|---|---|---|---|---|---|---|---|"]
    fmt = lambda v, f: "-" if v is None else format(v, f)  # noqa: E731
    for v, rs in sorted(rows.items()):
        for r in sorted(rs):
            out.append(f"| {v} | {r[0]} | {r[1]:.0f} | {r[2]:.4f} | {fmt(r[3], '.4f')} | {fmt(r[4], '.4f')} | "
                       f"{fmt(r[5], '.0f')} | {fmt(r[6], '.0f')} | {fmt(r[7], '.3f')} |")
        n = len(rs)
        mean = lambda i: sum(r[i] for r in rs if r[i] is not None) / max(1, sum(r[i] is not None for r in rs))  # noqa: E731
        out.append(f"| **{v}** | mean | {mean(1):.0f} | {mean(2):.4f} | {mean(3):.4f} | {mean(4):.4f} | {mean(5):.0f} | "
                   f"{mean(6):.0f} | |")
    txt = "\n".join(out) + "\n"
    print(txt)
    if len(sys.argv) > 2:
        os.makedirs(os.path.dirname(os.path.abspath(sys.argv[2])), exist_ok=True)
        open(sys.argv[2], "w").write(txt)


if __name__ == "__main__":
    main()
