#!/usr/bin/env python3
"""Where a kernel's scratch (spill) accesses sit: source line -> count of scratch_load/store, from a
-gline-tables-only device assembly (see tools/valu_lines.py for the build line).
Usage: spill_lines.py <kernel-substring> [asm]"""
import collections
import re
import sys

pat = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else "rust-ray-tracing_amd/build/dbg.s"
t = open(path).read()
name = next(m.group(1) for m in re.finditer(r"^(\S+):", t, re.M) if pat in m.group(1))
body = t[t.index(name + ":"):t.index(".Lfunc_end", t.index(name + ":"))].split("\n")
files = {m.group(1): m.group(3).split("/")[-1] for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]+)"', t)}
line = (0, "?")
cnt = collections.Counter()
for l in body:
    m = re.match(r"\s+\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        line = (int(m.group(2)), files.get(m.group(1), m.group(1)))
    elif re.match(r"\s+(scratch_|buffer_).*(load|store)", l) and ("scratch" in l or "off, s[0:3]" in l or "s[0:3]" in l):
        cnt[(line, "store" if "store" in l else "load")] += 1
for ((ln, f), k), c in sorted(cnt.items()):
    print(f"{f}:{ln:<5d} {k:5s} {c}")
