# E5 fp32 (K10) query encode under rocprofv3: per-kernel time of the graph replays
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/e5k; export TMPDIR=/tmp
E5_DTYPE=float32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/e5k/rp -o e5 --output-format csv -- python3 tools/e5_probe.py > gpurun_out/e5k/rp.log 2>&1 || { tail -20 gpurun_out/e5k/rp.log; exit 1; }
grep -E "graph|eager" gpurun_out/e5k/rp.log
f=$(find gpurun_out/e5k/rp -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/e5k/kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/e5k/kernel_stats.csv')))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:25]:
    print(f"{r['Name'][:90]:90s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:8.1f} tot_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
