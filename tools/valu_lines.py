#!/usr/bin/env python3
"""Static VALU/SALU/SMEM instruction counts per source line of one kernel instantiation.

Build the line-table assembly first:
  hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -std=c++17 -gline-tables-only --cuda-device-only \
        -S -o rust-ray-tracing_amd/build/dbg.s rust-ray-tracing_amd/csrc/rt_kernel.hip
Usage: valu_lines.py [kernel-substring] [first-line] [last-line] [asm] [source file, default rt_sweep.hpp]
"""
import collections
import re
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "trace_pathsIfLi5ELb0ELi0ELb1E"
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 1
hi = int(sys.argv[3]) if len(sys.argv) > 3 else 10 ** 9
path = sys.argv[4] if len(sys.argv) > 4 else "rust-ray-tracing_amd/build/dbg.s"
t = open(path).read()
files = {m.group(1): m.group(3) for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]+)"', t)}
name = next(m.group(1) for m in re.finditer(r"^(\S+):", t, re.M) if pat in m.group(1))
body = t[t.index(name + ":"):t.index(".Lfunc_end", t.index(name + ":"))].split("\n")
cnt = collections.defaultdict(collections.Counter)
cur = None
for line in body:
    s = line.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
    if m:
        cur = (files.get(m.group(1), "?"), int(m.group(2)))
        continue
    if not s or s.startswith((";", ".")) or s.endswith(":"):
        continue
    op = s.split()[0]
    k = "v" if op.startswith("v_") else "smem" if op.startswith("s_load") or op.startswith("s_buffer") else \
        "s" if op.startswith("s_") else "mem" if op.startswith(("global_", "ds_", "buffer_", "scratch_")) else "o"
    cnt[cur][k] += 1
srcf = sys.argv[5] if len(sys.argv) > 5 else "rt_sweep.hpp"
src = open("rust-ray-tracing_amd/csrc/" + srcf).read().split("\n")
tot = collections.Counter()
for c in cnt.values():
    tot.update(c)
print(name, dict(tot))
for (f, ln), c in sorted(((k, v) for k, v in cnt.items() if k), key=lambda x: (x[0][0], x[0][1])):
    if f.endswith(srcf) and lo <= ln <= hi:
        print(f"{ln:5d} v{c['v']:4d} s{c['s']:3d} m{c['smem'] + c['mem']:3d}  {src[ln - 1].strip()[:90]}")
