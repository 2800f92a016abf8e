#!/usr/bin/env python3
"""WRITE_SIZE / FETCH_SIZE calibration on gfx950 for the update kernel's access shapes (measurement tool).

  python tools/write_calib.py <dir> [out-prefix]

<dir> holds expected.json (tools/probes/build/write_calib's stdout) and the two rocprofv3 --pmc passes of that
binary, write/run_counter_collection.csv (WRITE_SIZE) and fetch/run_counter_collection.csv (FETCH_SIZE);
tools/gpu_session.sh step `calib` runs all three.  Writes <out-prefix>.json and <out-prefix>.md (default
profiles/r06/write_calib): per shape the counted bytes (KB x 1024) over the stored / loaded bytes and over the
32- / 64-B sectors touched.  bench.py reads the JSON for the update's roofline.traffic correction.
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path, name):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != name:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            out[k] = out.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0  # KB
    return out


def main():
    d = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r06", "write_calib")
    exp = json.loads([ln for ln in open(os.path.join(d, "expected.json")) if ln.startswith("{")][-1])
    wr = counters(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    fe = counters(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    rows = []
    for s in exp["shapes"]:
        k = s["kernel"]
        w, f = wr.get(k), fe.get(k)
        rows.append({
            "kernel": k, "bytes": s["bytes"], "sectors32_bytes": 32 * s["sectors32"], "sectors64_bytes": 64 * s["sectors64"],
            "write_size_bytes": w, "fetch_size_bytes": f,
            "write_over_bytes": w / s["bytes"] if w is not None else None,
            "write_over_sectors32": w / (32 * s["sectors32"]) if w is not None else None,
            "write_over_sectors64": w / (64 * s["sectors64"]) if w is not None else None,
            "fetch_x2_over_bytes": 2 * f / s["bytes"] if f is not None else None,
        })
    os.makedirs(os.path.dirname(prefix), exist_ok=True)
    with open(prefix + ".json", "w") as fo:
        json.dump({"shapes": rows, "source": "tools/probes/write_calib.hip, rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE "
                   "(one pass each)"}, fo, indent=1)
    fmt = lambda v: "—" if v is None else f"{v:.3f}"
    lines = ["# WRITE_SIZE / FETCH_SIZE calibration (gfx950, `tools/probes/write_calib.hip`)", "",
             "| shape | bytes stored / loaded | 32-B sectors touched (B) | WRITE_SIZE (B) | WRITE / bytes | WRITE / 32-B sectors "
             "| WRITE / 64-B sectors | 2 x FETCH / bytes |", "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{r['kernel']}` | {r['bytes']} | {r['sectors32_bytes']} | {r['write_size_bytes'] or 0:.0f} | "
                     f"{fmt(r['write_over_bytes'])} | {fmt(r['write_over_sectors32'])} | {fmt(r['write_over_sectors64'])} | "
                     f"{fmt(r['fetch_x2_over_bytes'])} |")
    open(prefix + ".md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
