#!/usr/bin/env python3
"""Per-kernel ISA statistics from a `hipcc --cuda-device-only -S` listing: VGPRs, LDS bytes,
flat / LDS / global / buffer instruction counts (flat accesses in a kernel that should address
LDS directly mean the address space was lost).
  python3 scripts/isa_stats.py file.s [name-substring ...]"""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
cur = None
stats = {}
for line in s.split("\n"):
    m = re.match(r"^(_Z\S+):\s", line)
    if m:
        cur = m.group(1)
        stats[cur] = {"flat": 0, "ds": 0, "global": 0, "buffer": 0, "lines": 0}
        continue
    if cur is None:
        continue
    if line.startswith(".Lfunc_end"):
        cur = None
        continue
    t = line.strip()
    for k in ("flat", "ds", "global", "buffer"):
        if t.startswith(k + "_"):
            stats[cur][k] += 1
    stats[cur]["lines"] += 1
for name, v in stats.items():
    if pats and not any(p in name for p in pats):
        continue
    vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", s)
    lds = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"\n(?:.*\n)*?\s+\.amdhsa_group_segment_fixed_size (\d+)", s)
    print(f"{name[:90]:90s} vgpr {vg.group(1) if vg else '?':>4s} lds {lds.group(1) if lds else '?':>6s} "
          + " ".join(f"{k} {v[k]}" for k in ("flat", "ds", "global", "buffer", "lines")))
