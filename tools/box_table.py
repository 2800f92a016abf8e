#!/usr/bin/env python3
"""Per-lease table of the driver's command lines under profiles/<round>/ (bench value, kernel times, the clock
probe's effective shader clock and cycles per workgroup, device-copy bandwidth):
    python3 tools/box_table.py r04 > profiles/r04/boxes.md"""
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r04"
    print(f"# Driver-command lines of round {rnd[1:]} (one lease each)\n")
    print("| file | streams | kernel_src | scans/s | ms/step | update ms | match ms | update MHz | match MHz | "
          "update kcycles/WG | match kcycles/WG | copy GB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", rnd, f"{rnd}*_driver_cmd*.json"))):
        d = json.load(open(f))
        r = d["roofline"]
        k = r["kernel_ms_per_step"]
        cp = r.get("clock_probe") or {}
        cu = (cp.get("update") or {}).get("cycles_per_workgroup")
        cm = (cp.get("match") or {}).get("cycles_per_workgroup")
        print(f"| {os.path.basename(f)} | {d['config']['streams_per_gpu']} | {d['config'].get('kernel_src')} | "
              f"{d['value']:.0f} | {d['ms_per_step']:.4f} | {k['update']:.4f} | {k['match']:.4f} | "
              f"{r.get('update_sclk_mhz')} | {r.get('match_sclk_mhz')} | {cu / 1e3 if cu else '—'} | "
              f"{cm / 1e3 if cm else '—'} | {r.get('attainable_copy_GBps')} |")


if __name__ == "__main__":
    main()
