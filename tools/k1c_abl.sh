#!/bin/bash
# GPU: K1c timing ablations, compile-time (variants/lib_d<bits>.so built with -DK1C_DBG=<bits>):
#   0 full kernel | 1024 no DMA issue (compute side) | 4096 no MFMA (memory side) | 128 no epilogue
#   | 512 no barrier (races; timing only)
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do for f in variants/lib_*.so; do
  CLASSMATE_HIP_LIB=$PWD/$f timeout -k 10 300 python tools/dense_probe.py --reps 7 2>&1 | grep docs= | sed "s/^/$(basename $f .so) /" | cut -c1-120
done; done
