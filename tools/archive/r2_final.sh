#!/bin/bash
# GPU (round-2 evidence, part 1): every -m gpu test (BASELINE-size ones included), smoke, fresh PMC
# traffic of K2a, and a kernel-trace profile of the headline bench.  Each GPU step under its own
# limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r02v2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/pytest_${R}.log 2>&1 || { tail -30 gpurun_out/pytest_${R}.log; exit 1; }
tail -2 gpurun_out/pytest_${R}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${R}.log 2>&1 || { tail -20 gpurun_out/smoke_${R}.log; exit 1; }
tail -1 gpurun_out/smoke_${R}.log
ROUND=$R ONLY="${PMC_ONLY:-bm25_B256}" bash tools/pmc_traffic.sh || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${R} -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline 0 --e5-fp32-leg 0 > gpurun_out/prof_${R}.log 2>&1 || { tail -20 gpurun_out/prof_${R}.log; exit 1; }
f=$(find gpurun_out/prof_${R} -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${R}_hybrid_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  calls={r["Calls"]:>5}  avg={float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
