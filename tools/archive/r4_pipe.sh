#!/bin/bash
# GPU: headline A/B -- serial step vs --pipeline 1 (encode of batch i+1 beside batch i's search), recall check on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/pipe; export TMPDIR=/tmp
HL="--steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0"
for rep in 1 2; do for v in 0 2; do
  timeout -k 10 300 python -u bench.py $HL --pipeline $v --cpu-baseline $([ $rep = 1 ] && echo 1 || echo 0) --out gpurun_out/pipe/b_$v$rep.json > gpurun_out/pipe/b_$v$rep.log 2>&1 || { tail -30 gpurun_out/pipe/b_$v$rep.log; exit 1; }
  echo "pipe=$v $(python -c "import json;d=json.load(open('gpurun_out/pipe/b_$v$rep.json'));print(d['value'],d['ms_per_step'],d['breakdown_ms'],d.get('recall_at_10',d.get('recall')))")" | tee -a gpurun_out/pipe/ab.txt
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pipe/trace -o hl --output-format csv -- python3 -u bench.py $HL --cpu-baseline 0 --pipeline 2 --out gpurun_out/pipe/b_tr.json > gpurun_out/pipe/tr.log 2>&1 || { tail -30 gpurun_out/pipe/tr.log; exit 1; }
grep "steps in" gpurun_out/pipe/tr.log | cut -c1-200
