#!/bin/bash
# GPU: K1q seed-sample fraction A/B (CM_K1Q_SAMPLE = 16 product / 32 / 24) on the headline step + the standalone
# dense probe (B = 256, k = 24 at 10M)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/smp; export TMPDIR=/tmp
HL="--steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0"
for rep in 1 2; do for s in 16 32 24; do
  CM_K1Q_SAMPLE=$s timeout -k 10 300 python -u bench.py $HL --out gpurun_out/smp/b_$s$rep.json > gpurun_out/smp/b.log 2>&1 || { tail -30 gpurun_out/smp/b.log; exit 1; }
  echo "sample=1/$s $(python -c "import json;d=json.load(open('gpurun_out/smp/b_$s$rep.json'));print(round(d['value']),round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['breakdown_ms'].items()},d['dense_exact_reruns'])")" | tee -a gpurun_out/smp/ab.txt
done; done
for s in 16 32 24 16 32 24; do
  CM_K1Q_SAMPLE=$s timeout -k 10 300 python tools/dense_probe.py --reps 7 > gpurun_out/smp/p.log 2>&1 || { tail -20 gpurun_out/smp/p.log; exit 1; }
  grep docs= gpurun_out/smp/p.log | sed "s/^/sample=1\/$s /" | cut -c1-160 | tee -a gpurun_out/smp/ab.txt
done
