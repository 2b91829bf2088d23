#!/usr/bin/env python3
"""Timeline of one decode step from a rocprofv3 kernel trace: per kernel duration and the
gap to the previous kernel's end (graph-launched chain)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", n.replace("void ", "").replace("mtts::", ""))[:48]
# find decode steps: sequences starting at embed_kernel
idx = [i for i, r in enumerate(rows) if "embed_kernel" in r["Kernel_Name"]]
step = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
a, b = idx[step], idx[step + 1]
tot_gap = defaultdict(float)
tot_dur = defaultdict(float)
cnt = defaultdict(int)
prev_end = None
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    n = short(r["Kernel_Name"]) + f" g{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    gap = (s - prev_end) / 1000 if prev_end else 0.0
    tot_gap[n] += gap
    tot_dur[n] += (e - s) / 1000
    cnt[n] += 1
    prev_end = e
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1000
print(f"step {step}: span {span:.1f} us, kernels {b - a}")
for n in sorted(tot_dur, key=lambda k: -tot_dur[k]):
    print(f"  {n:70s} n={cnt[n]:3d} dur/call {tot_dur[n] / cnt[n]:7.2f}  gap/call {tot_gap[n] / cnt[n]:6.2f}")
print(f"  total dur {sum(tot_dur.values()):.1f}  total gap {sum(tot_gap.values()):.1f}")
# in-order listing of the step's first kernels (one layer and the lead-in): KTRACE_SEQ=N
import os
nseq = int(os.environ.get("KTRACE_SEQ", "0"))
for r in rows[a:a + nseq]:
    print(f"    {short(r['Kernel_Name']):48s} g{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
          f"  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000:7.2f} us")
