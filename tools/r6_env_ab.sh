#!/bin/bash
# Round 6: same-box A/B of environment knobs in the headline step (no side legs), alternating.
# ENVS="name=VAR=val,VAR2=val2 name2=..." (name "base" = no knob); REPS rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/envab; export TMPDIR=/tmp
ENVS=${ENVS:-"base full=CM_DENSE_F16=full q8seed=CM_K1Q_SEED=q8"}
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $ENVS; do
    name=${spec%%=*}; kv=""; [ "$spec" != "$name" ] && kv=${spec#*=}
    envs=(); IFS=',' read -ra parts <<< "$kv"; for p in "${parts[@]}"; do [ -n "$p" ] && envs+=("$p"); done
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --dense-legs 0 --e5-other-leg 0 \
      --ingest-leg 0 --cpu-baseline 0 --out gpurun_out/envab/${name}_$rep.json > gpurun_out/envab/${name}_$rep.log 2>&1 \
      || { echo "$name failed"; tail -20 gpurun_out/envab/${name}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/${name}_$rep.json'));print('$name', round(d['value']), {k:round(x,3) for k,x in d['breakdown_ms'].items() if x})"
  done
done
