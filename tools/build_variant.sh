#!/bin/bash
# build_variant.sh NAME "EXTRA HIPCC FLAGS" -> variants/lib_NAME.so (K2 compile-time knobs, for A/B probes)
set -e
cd "$(dirname "$0")/../classmate-rag_amd"
make -s -j4 >/dev/null
SRC=${SRC:-csrc}   # SRC=dir holding an alternative cm_bm25.hip + cm_bm25_prune.inc (e.g. from git show)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off ${NOABL:+-UCM_ABLATION}${NOABL:--DCM_ABLATION} $2 -I../include -Icsrc -c $SRC/cm_bm25.hip -o build/cm_bm25_$1.o
mkdir -p ../variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/lib_$1.so build/cm_api.o build/cm_bm25_$1.o build/cm_dense.o build/cm_fusion.o build/cm_pool.o build/cm_filter.o build/cm_encoder.o build/cm_gemm.o
