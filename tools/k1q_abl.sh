#!/bin/bash
# GPU: K1q timing ablations (variants/lib_q<bits>.so built with -DK1Q_DBG=<bits>), forced kind 5:
#   product | 64 no appends | 128 no epilogue | 1024 no DMA in the loop (compute side) | 4096 no MFMA
#   (memory side) | 8192 L2-resident source | 5120 = 1024 + 4096 (loop skeleton: barriers, reads)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/q8abl
for rep in 1 2; do for f in classmate-rag_amd/classmate_hip/libclassmate_hip.so variants/lib_q*.so; do
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/q8abl/one.log 2>&1 || { tail -20 gpurun_out/q8abl/one.log; exit 1; }
  grep docs= gpurun_out/q8abl/one.log | sed "s/^/$(basename $f .so) /" | cut -c1-150 | tee -a gpurun_out/q8abl/abl.txt
done; done
