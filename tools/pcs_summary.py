#!/usr/bin/env python3
"""Aggregate a rocprofv3 PC-sampling CSV (host_trap) by instruction: samples per code-object offset,
with the instruction text, heaviest first.  Usage: pcs_summary.py <csv> [top]"""
import csv
import collections
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 400
with open(path, newline="") as f:
    r = csv.DictReader(f)
    cols = r.fieldnames
    print("columns:", cols)
    off = next((c for c in cols if "offset" in c.lower()), None)
    ins = next((c for c in cols if "instruction" in c.lower() and "comment" not in c.lower()), None)
    com = next((c for c in cols if "comment" in c.lower()), None)
    kern = next((c for c in cols if "kernel" in c.lower() or "dispatch" in c.lower()), None)
    cnt = collections.Counter()
    text = {}
    n = 0
    for row in r:
        n += 1
        k = (row.get(off) if off else "?")
        cnt[k] += 1
        if k not in text:
            text[k] = (row.get(ins, "") if ins else "", row.get(com, "") if com else "")
print("samples", n)
acc = 0
for k, v in cnt.most_common(top):
    acc += v
    t, c = text[k]
    print(f"{v:8d} {100.0 * v / n:6.2f}% {100.0 * acc / n:6.1f}%  {k:>10}  {t:60s} {c[-90:]}")
