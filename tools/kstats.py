#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace directory: per kernel name calls / avg / min / max / total,
computed from the per-launch kernel_trace.csv (so the summary can also be split by launch grid)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'tot_ms':>9s}")
for name, v in out:
    print(f"{name[:90]:90s} {len(v):6d} {sum(v)/len(v):9.1f} {min(v):9.1f} {max(v):9.1f} {sum(v)/1e3:9.2f}")
