#!/bin/bash
# GPU: the round's bench lines (headline hybrid, C2 1M x 768 B=256, C2' 10M B=16) and a kernel-trace
# profile of the headline run.  Each step under its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r02}
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --out gpurun_out/bench_${R}_hybrid.json > gpurun_out/bench_${R}_hybrid.log 2>&1 || { tail -20 gpurun_out/bench_${R}_hybrid.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_${R}_hybrid.log
timeout -k 10 300 python -u bench.py --mode dense --docs-per-gpu 1000000 --batch 256 --k 10 --steps 50 --warmup 5 --out gpurun_out/bench_${R}_c2_1m_b256.json > gpurun_out/bench_${R}_c2.log 2>&1 || { tail -20 gpurun_out/bench_${R}_c2.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_${R}_c2.log
timeout -k 10 300 python -u bench.py --mode dense --docs-per-gpu 10000000 --batch 16 --k 10 --steps 50 --warmup 5 --out gpurun_out/bench_${R}_c2p_10m_b16.json > gpurun_out/bench_${R}_c2p.log 2>&1 || { tail -20 gpurun_out/bench_${R}_c2p.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_${R}_c2p.log
[ "${PROF:-1}" = "1" ] || exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R} -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --e5-fp32-leg 0 > gpurun_out/prof_${R}.log 2>&1 || { tail -20 gpurun_out/prof_${R}.log; exit 1; }
f=$(find gpurun_out/prof_${R} -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${R}_hybrid_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  calls={r["Calls"]:>5}  avg={float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
