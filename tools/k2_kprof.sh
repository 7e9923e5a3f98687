#!/bin/bash
# GPU: kernel trace of the 10M BM25 probe (pruned path) for the product library and each
# variants/lib_*.so; prints the per-search kernels' average durations side by side.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in product ${VARIANTS:-variants/lib_*.so}; do
  n=$(basename $v .so)
  if [ "$v" = product ]; then unset CLASSMATE_HIP_LIB; else export CLASSMATE_HIP_LIB=$PWD/$v; fi
  rm -rf gpurun_out/kp_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kp_$n -o kp --output-format csv -- python3 tools/bm25_probe.py --paths 2 --reps 7 > gpurun_out/kp_$n.log 2>&1 || { tail -20 gpurun_out/kp_$n.log; exit 1; }
  f=$(find gpurun_out/kp_$n -name '*kernel_stats.csv' | head -1)
  echo "== $n $(grep -o 'search_ms=[0-9.]*' gpurun_out/kp_$n.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r['Calls']) in (8, 16) and 'cm::' in r['Name']:
        print(f"  {r['Name'][:48]:48s} calls={r['Calls']:>3s} avg_us={float(r['AverageNs'])/1e3:8.1f}")
PY
done
