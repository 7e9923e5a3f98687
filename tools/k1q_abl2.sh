#!/bin/bash
# GPU: K1q epilogue split (variants/lib_q<bits>.so, -DK1Q_DBG=<bits>), forced kind 5, Gaussian probe queries:
#   product | q64: hit tests kept alive, no appends | q128: no epilogue | any other variants/lib_*.so
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/q8abl2
for rep in 1 2; do for f in classmate-rag_amd/classmate_hip/libclassmate_hip.so variants/lib_*.so; do
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --path 5 --reps 7 > gpurun_out/q8abl2/one.log 2>&1 || { tail -20 gpurun_out/q8abl2/one.log; exit 1; }
  grep docs= gpurun_out/q8abl2/one.log | sed "s/^/$(basename $f .so) /" | cut -c1-150 | tee -a gpurun_out/q8abl2/abl.txt
done; done
