#!/bin/bash
# Register / LDS / spill summary of the Hector kernels from the device assembly (CPU only, no GPU):
#   tools/kstats.sh [extra hipcc flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/creating-2d-laser-slam-from-scratch_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    --cuda-device-only -S hector_capi.hip -o /tmp/hector_kstats.s "$@" 2>/dev/null || exit 1
python3 - <<'PY'
import re
txt = open("/tmp/hector_kstats.s").read()
for blk in re.findall(r"  - \.agpr_count.*?(?=\n  - \.agpr_count|\namdhsa\.target|\Z)", txt, flags=re.S):
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = g("name")
    if "hs_" not in name:
        continue
    short = re.sub(r"^_ZN3s2d\d+", "", name)[:40]
    print(f"{short:42s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} vspill {g('vgpr_spill_count'):>3} "
          f"sspill {g('sgpr_spill_count'):>3} lds {g('group_segment_fixed_size'):>6} priv {g('private_segment_fixed_size'):>4}")
PY
