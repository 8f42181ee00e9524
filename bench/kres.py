#!/usr/bin/env python3
"""Register / LDS / spill summary per kernel from a gfx950 .s file (amdhsa metadata).
usage: python bench/kres.py FILE.s [name-substring]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
meta = s[s.index("amdhsa.kernels:"):]
for ent in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", ent))
    if sub in f.get("name", ""):
        print(f"{f.get('name','?')[:90]:90s} vgpr={f.get('vgpr_count')} agpr={f.get('agpr_count')} "
              f"spill={f.get('vgpr_spill_count')} lds={f.get('group_segment_fixed_size')}")
