#!/usr/bin/env python3
"""Per-kernel register usage from the device assembly (make -C rust-ray-tracing_amd asm)."""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "rust-ray-tracing_amd/build/rt_kernel-gfx950.s"
pat = sys.argv[2] if len(sys.argv) > 2 else "trace_paths"
t = open(path).read()
meta = t[t.index("amdhsa.kernels:"):]
for e in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", e)
    if not name or pat not in name.group(1):
        continue
    g = {k: (re.search(r"\." + k + r":\s+(\d+)", e) or [None, "?"])[1]
         for k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count")}
    print(f"{name.group(1):60s} v{g['vgpr_count']:>4} a{g['agpr_count']:>3} s{g['sgpr_count']:>4} "
          f"vspill {g['vgpr_spill_count']:>3} sspill {g['sgpr_spill_count']:>3}")
