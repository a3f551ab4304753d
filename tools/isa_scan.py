#!/usr/bin/env python3
"""Dev tool: per kernel, the memory instructions of a hipcc -S -gline-tables-only listing by source
line (flat_* = a generic pointer that lost its address space; global_load of a __constant__ table
inside a per-block chain = a vector memory round trip).
    python tools/isa_scan.py LISTING.s [KERNEL_SUBSTRING] [PATTERN]"""
import collections
import re
import sys

path = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else ""
pat = re.compile(sys.argv[3] if len(sys.argv) > 3 else r"(flat_\w+|global_load\w*|buffer_load\w*)")
files, cnt, cur, fn = {}, collections.Counter(), None, None
for line in open(path):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        fn = m.group(1)
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', line)
    if m:
        files[m.group(1)] = m.group(2).split("/")[-1]
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
    if m:
        cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
        continue
    m = re.match(r"\s+(\w+)", line)
    if m and fn and ksub in fn and pat.fullmatch(m.group(1)):
        cnt[(fn[:40], m.group(1), cur)] += 1
for k, v in sorted(cnt.items(), key=lambda kv: (kv[0][0], -kv[1])):
    print(v, k)
