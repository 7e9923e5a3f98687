#!/bin/bash
# GPU: dense K1 timing + kernel trace + HBM traffic (FETCH_SIZE, separate pass).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/dense_probe.py > gpurun_out/dprobe.log 2>&1 || { tail -20 gpurun_out/dprobe.log; exit 1; }
tail -1 gpurun_out/dprobe.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/dpmc -o pmc --output-format csv -- python3 tools/dense_probe.py --reps 2 > gpurun_out/dpmc.log 2>&1 || { tail -20 gpurun_out/dpmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/dpmc/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r['Kernel_Name'][:60]].append(float(r['Counter_Value']))
for k, v in agg.items():
    if 'dense' in k:
        print(k, 'launches', len(v), 'FETCH_SIZE KB/launch avg', sum(v) / len(v))
PY
