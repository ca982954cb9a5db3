"""Summarise a rocprofv3 kernel trace: mean duration per kernel and the idle gap before each kernel
(start minus the previous kernel's end on the same queue), over the last steps of the bench."""
import csv
import glob
import sys
from collections import defaultdict

path = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:]  # skip setup / warmup
dur, gap = defaultdict(list), defaultdict(list)
prev_end = None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].split("<")[0][-40:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[name].append((e - s) / 1e3)
    if prev_end is not None and 0 <= s - prev_end < 50_000:
        gap[name].append((s - prev_end) / 1e3)
    prev_end = e
for k in dur:
    g = gap.get(k, [])
    print(f"{k:42s} n={len(dur[k]):5d} dur={sum(dur[k]) / len(dur[k]):8.2f} us  gap_before={sum(g) / max(1, len(g)):6.2f} us")
