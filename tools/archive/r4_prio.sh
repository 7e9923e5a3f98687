#!/bin/bash
# GPU: step schedule A/B -- K1q LDS 160 KiB (product) vs 131 KiB (variants/lib_lds131.so: BM25 blocks fit beside
# it) x BM25 stream priority 0 / -1 (high)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/prio; export TMPDIR=/tmp
HL="--steps 20 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0"
for rep in 1 2; do for lib in prod lds131; do for pr in 0 -1; do
  if [ $lib = prod ]; then L=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; else L=$PWD/variants/lib_$lib.so; fi
  CLASSMATE_HIP_LIB=$L timeout -k 10 300 python -u bench.py $HL --bm25-priority $pr --out gpurun_out/prio/b.json > gpurun_out/prio/b.log 2>&1 || { tail -30 gpurun_out/prio/b.log; exit 1; }
  echo "$lib prio=$pr $(python -c "import json;d=json.load(open('gpurun_out/prio/b.json'));print(round(d['value']),round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['breakdown_ms'].items()})")" | tee -a gpurun_out/prio/ab.txt
done; done; done
