#!/usr/bin/env python3
"""VGPR / SGPR / scratch / LDS per kernel from a hipcc -save-temps .s file."""
import re
import sys

s = open(sys.argv[1]).read()
meta = s[s.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or "k_" not in name.group(1):
        continue
    g = lambda k: (re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "?"])[1]
    print("%-70s vgpr %4s sgpr %4s scratch %4s lds %6s" % (
        name.group(1)[:70], g("vgpr_count"), g("sgpr_count"),
        g("private_segment_fixed_size"), g("group_segment_fixed_size")))
