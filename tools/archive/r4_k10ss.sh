#!/bin/bash
# GPU: ring depth of the K10 64 x 32 tile (M <= 32): product (4 stages) vs variants/lib_k10_s6 / s8 -- batch-1 E5 latency, twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k10ss
for rep in 1 2; do for v in prod s6 s8; do
  if [ $v = prod ]; then L=$PWD/classmate-rag_amd/classmate_hip/libclassmate_hip.so; else L=$PWD/variants/lib_k10_$v.so; fi
  CLASSMATE_HIP_LIB=$L timeout -k 10 200 python -u tools/e5_b1_probe.py > gpurun_out/k10ss/p.log 2>&1 || { tail -20 gpurun_out/k10ss/p.log; exit 1; }
  grep "B=1:" gpurun_out/k10ss/p.log | sed "s/^/$v /" | tee -a gpurun_out/k10ss/ab.txt
done; done
