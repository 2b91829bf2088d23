#!/usr/bin/env python3
"""Per-frame breakdown of a MossTTSLocal decode from a rocprofv3 kernel trace (csv): frames
are delimited by local_finalize_kernel; reports the mean frame span, busy time, and the
per-frame duration / count / idle gap per kernel over the middle frames."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", n.replace("void ", "").replace("mtts::", ""))[:60]
ends = [i for i, r in enumerate(rows) if "local_finalize_kernel" in r["Kernel_Name"]]
sel = list(zip(ends[2:-2], ends[3:-1]))  # skip the prefill frame and warm-up edges
dur, gap, cnt = defaultdict(float), defaultdict(float), defaultdict(int)
span = busy = 0.0
for a, b in sel:
    prev = int(rows[a]["End_Timestamp"])
    span += (int(rows[b]["End_Timestamp"]) - prev) / 1e3
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        n = short(r["Kernel_Name"])
        dur[n] += (e - s) / 1e3
        gap[n] += (s - prev) / 1e3
        cnt[n] += 1
        busy += (e - s) / 1e3
        prev = e
F = max(len(sel), 1)
print(f"frames {F}: span {span / F:.1f} us/frame, busy {busy / F:.1f} us, idle {(span - busy) / F:.1f} us, "
      f"kernels/frame {sum(cnt.values()) / F:.0f}")
print(f"{'kernel':60s} {'us/frame':>9s} {'calls':>6s} {'us/call':>8s} {'gap us':>8s}")
for n in sorted(dur, key=lambda k: -dur[k]):
    print(f"{n:60s} {dur[n] / F:9.1f} {cnt[n] / F:6.0f} {dur[n] / cnt[n]:8.2f} {gap[n] / F:8.1f}")
