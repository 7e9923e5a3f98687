#!/bin/bash
# GPU: K2a tf-slot packing A/B (variants/lib_pk0 = one register per slot, pk1 = packed pairs, pk1w6 = packed at 6
# waves/SIMD): 10M BM25 pruned search, identity against the full K2 scan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out/k2a
VARS="pk0 pk1 pk1w6 pk0 pk1 pk1w6" bash tools/ab_bm25.sh 2>&1 | tee gpurun_out/k2a/ab.txt
