#!/bin/bash
# GPU: K1q LDS budget A/B in the headline step (160 KiB product vs variants/lib_*.so), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/ldsab; export TMPDIR=/tmp
for rep in 1 2; do for f in classmate-rag_amd/classmate_hip/libclassmate_hip.so variants/lib_*.so; do
  n=$(basename $f .so)
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --e5-other-leg 0 --ingest-leg 0 --dense-legs 0 --cpu-baseline 0 --out gpurun_out/ldsab/$n.json > gpurun_out/ldsab/$n.log 2>&1 || { tail -20 gpurun_out/ldsab/$n.log; exit 1; }
  echo "$n $(grep 'steps in' gpurun_out/ldsab/$n.log | cut -c1-200)"
done; done
