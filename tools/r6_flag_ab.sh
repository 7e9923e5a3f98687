#!/bin/bash
# Round 6: same-box A/B of bench.py flag sets in the headline step (no side legs), alternating.
# FLAGS="name:--flag v --flag2 v;name2:..." (name base = product defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/flagab; export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${FLAGS:-base:;gate2:--bm25-gate 2}"
for rep in $(seq 1 ${REPS:-2}); do
  for set in "${SETS[@]}"; do
    name=${set%%:*}; fl=${set#*:}
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --dense-legs 0 --e5-other-leg 0 --ingest-leg 0 \
      --cpu-baseline 0 $fl --out gpurun_out/flagab/${name}_$rep.json > gpurun_out/flagab/${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -20 gpurun_out/flagab/${name}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/flagab/${name}_$rep.json'));print('$name', round(d['value']), {k:round(x,3) for k,x in d['breakdown_ms'].items() if x})"
  done
done
