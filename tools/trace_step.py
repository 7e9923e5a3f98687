"""Print one step's kernel timeline (kernels > MIN us) from a rocprofv3 kernel-trace CSV: the step is
anchored on the last launch of ANCHOR (default: the dense scan).  usage: trace_step.py CSV [ANCHOR] [MIN_US]"""
import collections
import csv
import sys

path = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "dense_q8_scan_kernel"
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 20.0
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
last = [r for r in rows if anchor in r["Kernel_Name"]][-1]
t0 = int(last["Start_Timestamp"]) - 5_000_000
for r in rows:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    if 0 < s < 14000 and e - s > min_us:
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r.get('Queue_Id', '')} {r['Kernel_Name'][:70]}")
