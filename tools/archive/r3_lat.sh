#!/bin/bash
# single-query retrieve() latency breakdown: kernel trace of the e2e bench at 1M chunks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/lat; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/lat/rp -o lat --output-format csv -- python3 -u bench.py --mode e2e --docs-per-gpu 1000000 --steps 5 --warmup 2 --out gpurun_out/lat/e2e.json > gpurun_out/lat/e2e.log 2>&1 || { tail -30 gpurun_out/lat/e2e.log; exit 1; }
grep -E "retrieve_batch calls" gpurun_out/lat/e2e.log | tail -1
f=$(find gpurun_out/lat/rp -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
# the last 20 retrieve() calls: group kernels into calls by gaps > 300 us
segs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b['Start_Timestamp']) - int(a['End_Timestamp']) > 300000: segs.append(cur); cur = [b]
    else: cur.append(b)
segs.append(cur)
for s in segs[-3:]:
    t0, t1 = int(s[0]['Start_Timestamp']), int(s[-1]['End_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in s)
    print(f"call: {len(s)} kernels, span {(t1-t0)/1e3:.1f} us, busy {busy/1e3:.1f} us")
s = segs[-1]
agg = collections.defaultdict(lambda: [0, 0])
for r in s:
    n = r['Kernel_Name'][:70]; agg[n][0] += 1; agg[n][1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"  {n:70s} {c:4d} {t/1e3:8.1f} us")
PY
