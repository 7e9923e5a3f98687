#!/bin/bash
# build_bm25_variant.sh NAME "EXTRA HIPCC FLAGS" -> variants/lib_NAME.so (cm_bm25.hip compile-time knobs, A/B probes)
set -e
cd "$(dirname "$0")/../classmate-rag_amd"
make -s -j8 >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $2 -I../include -Icsrc -c csrc/cm_bm25.hip -o build/cm_bm25_$1.o
mkdir -p ../variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/lib_$1.so build/cm_api.o build/cm_dense.o build/cm_bm25_$1.o build/cm_fusion.o build/cm_pool.o build/cm_filter.o build/cm_encoder.o build/cm_gemm.o
