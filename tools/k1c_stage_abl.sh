#!/bin/bash
# GPU: how much of K1c's scan is the in-loop candidate stores (K1C_NOHIT: never append) and does a
# 6-slot ring (room for LDS staging) cost anything -- tools/dense_probe.py --path 3, 10M x 768, B = 256
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k1cst
for rep in 1 2; do for f in classmate-rag_amd/classmate_hip/libclassmate_hip.so variants/lib_k1c_*.so; do
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --path 3 --reps 7 > gpurun_out/k1cst/one.log 2>&1 || { tail -20 gpurun_out/k1cst/one.log; exit 1; }
  grep docs= gpurun_out/k1cst/one.log | sed "s/^/$(basename $f .so) /" | cut -c1-150 | tee -a gpurun_out/k1cst/abl.txt
done; done
