#!/usr/bin/env python3
"""Instruction mix of kernels in a hipcc -save-temps .s file.
usage: python3 tools/isa_mix.py file.s <symbol-substring> [top]"""
import re
import sys
from collections import Counter

path, sub = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
cur, body = None, {}
for line in open(path):
    m = re.match(r"^(_Z\S+):", line)
    if m:
        cur = m.group(1) if sub in m.group(1) else None
        if cur:
            body[cur] = []
        continue
    if cur is not None:
        if "s_endpgm" in line:
            body[cur].append("s_endpgm")
            cur = None
            continue
        m = re.match(r"^\s+([a-z_][a-z0-9_]*)", line)
        if m:
            body[cur].append(m.group(1))
meta = {}
for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?", open(path).read()):
    pass
for k, ins in body.items():
    c = Counter(ins)
    print(f"{k[-70:]}: {len(ins)} instrs | " + " ".join(f"{n}:{v}" for n, v in c.most_common(top)))
