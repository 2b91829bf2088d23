#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: share, calls, average duration per kernel."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:6.2f}% calls={r['Calls']:>7} avg_us={float(r['AverageNs']) / 1e3:9.2f} "
          f"min_us={float(r['MinNs']) / 1e3:8.2f} {r['Name'][:90]}")
print("total ms", round(tot / 1e6, 2))
