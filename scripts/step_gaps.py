#!/usr/bin/env python3
"""Idle time between decode steps from a rocprofv3 kernel trace (csv): steps are delimited by
embed_kernel launches; for the middle steps reports the mean busy time, the mean gap before a
step's first kernel (graph-to-graph), the gaps inside a step, and the largest gaps (poll
bubbles every `chunk` steps show up there).
  python3 scripts/step_gaps.py kernel_trace.csv [max kernels per step, default 20]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "embed_kernel" in r["Kernel_Name"]]
# decode steps: consecutive embed launches with a single-token grid (prefill embeds are larger)
steps = []
for a, b in zip(idx, idx[1:]):
    if b - a < (int(sys.argv[2]) if len(sys.argv) > 2 else 20):
        steps.append((a, b))
steps = steps[5:-5]
inter, intra, busy, big = [], [], [], []
for a, b in steps:
    s0 = int(rows[a]["Start_Timestamp"])
    prev_end = int(rows[a - 1]["End_Timestamp"])
    inter.append((s0 - prev_end) / 1e3)
    bz, gp = 0.0, 0.0
    pe = None
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        bz += (e - s) / 1e3
        if pe is not None:
            gp += max(0, s - pe) / 1e3
        pe = e
    busy.append(bz)
    intra.append(gp)
n = len(steps)
inter_sorted = sorted(inter)
print(f"steps {n}: busy {sum(busy) / n:.1f} us/step, gaps inside a step {sum(intra) / n:.2f} us, "
      f"gap before a step: mean {sum(inter) / n:.2f} us, median {inter_sorted[n // 2]:.2f}, "
      f"max {inter_sorted[-1]:.1f}")
print("largest gaps before a step (us):", [round(x, 1) for x in inter_sorted[-12:]])
print(f"share of the steps' wall time idle: {(sum(inter) + sum(intra)) / (sum(inter) + sum(intra) + sum(busy)):.4f}")
